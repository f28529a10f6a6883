// Minimal fake librocm_smi64.so.1 (memory queries only) for CPU tests of the
// rocm-smi virtualisation in the enforcement library (native/shim/hooks_rsmi.cpp).
// Every device reports VGPU_FAKE_MEM bytes of VRAM (default 288 GiB) and
// VGPU_FAKE_RSMI_USED bytes in use.
#include <rocm_smi/rocm_smi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t env_u64(const char* n, uint64_t d) {
  const char* v = getenv(n);
  return v && *v ? strtoull(v, nullptr, 10) : d;
}

extern "C" {

rsmi_status_t rsmi_init(uint64_t) { return RSMI_STATUS_SUCCESS; }
rsmi_status_t rsmi_shut_down(void) { return RSMI_STATUS_SUCCESS; }
rsmi_status_t rsmi_num_monitor_devices(uint32_t* n) {
  *n = (uint32_t)env_u64("VGPU_FAKE_GPUS", 1);
  return RSMI_STATUS_SUCCESS;
}
rsmi_status_t rsmi_dev_memory_total_get(uint32_t, rsmi_memory_type_t, uint64_t* total) {
  *total = env_u64("VGPU_FAKE_MEM", 288ull << 30);
  return RSMI_STATUS_SUCCESS;
}
rsmi_status_t rsmi_dev_memory_usage_get(uint32_t, rsmi_memory_type_t, uint64_t* used) {
  *used = env_u64("VGPU_FAKE_RSMI_USED", 1ull << 30);
  return RSMI_STATUS_SUCCESS;
}

// VGPU_FAKE_RSMI_BDFS="dddd:bb:dd.f,...": PCI address of each rsmi index
// (default 0000:<0x05 + 0x10 i>:00.0, the fake node's layout).
rsmi_status_t rsmi_dev_pci_id_get(uint32_t dv, uint64_t* id) {
  if (!id) return RSMI_STATUS_INVALID_ARGS;
  if (dv >= (uint32_t)env_u64("VGPU_FAKE_GPUS", 1)) return RSMI_STATUS_INVALID_ARGS;
  unsigned dom = 0, bus = 0x05 + 0x10 * dv, dev = 0, fn = 0;
  if (const char* v = getenv("VGPU_FAKE_RSMI_BDFS")) {
    const char* p = v;
    for (uint32_t i = 0; i < dv && p; ++i) {
      p = strchr(p, ',');
      if (p) ++p;
    }
    if (p) sscanf(p, "%x:%x:%x.%x", &dom, &bus, &dev, &fn);
  }
  *id = ((uint64_t)dom << 32) | (bus << 8) | (dev << 3) | fn;
  return RSMI_STATUS_SUCCESS;
}

// VGPU_FAKE_RSMI_PIDS="pid,pid,..": compute processes on the "node".
rsmi_status_t rsmi_compute_process_info_get(rsmi_process_info_t* procs, uint32_t* num) {
  const char* v = getenv("VGPU_FAKE_RSMI_PIDS");
  uint32_t n = 0;
  for (const char* p = v; p && *p;) {
    char* end;
    unsigned long pid = strtoul(p, &end, 10);
    if (end == p) break;
    if (procs && n < *num) procs[n] = rsmi_process_info_t{(uint32_t)pid, 0, 1ull << 20, 0, 0};
    ++n;
    p = *end ? end + 1 : end;
  }
  const bool small = procs && n > *num;
  *num = n;
  return small ? RSMI_STATUS_INSUFFICIENT_SIZE : RSMI_STATUS_SUCCESS;
}

}  // extern "C"
