// rocm-smi (librocm_smi64) memory virtualisation — the rocm-smi twin of
// hooks_smi.cpp (reference: nvmlDeviceGetMemoryInfo).
// rsmi device indices are the container-visible ordinals.
#include <rocm_smi/rocm_smi.h>

#include <algorithm>
#include <vector>

#include "common.h"
#include "real.h"
#include "state.h"

using namespace vgpu;

#define REAL_RSMI(name) \
  ((decltype(&::name))smi_real(#name, __builtin_return_address(0), rsmi_lib_handle))

static bool rsmi_vram(rsmi_memory_type_t t) {
  return t == RSMI_MEM_TYPE_VRAM || t == RSMI_MEM_TYPE_VIS_VRAM;
}

static uint64_t rsmi_limit(uint32_t dv) {
  ensure_init();
  if (!st().enabled || dv >= VGPU_MAX_DEVICES) return 0;
  return mem_limit((int)dv);
}

extern "C" {

__attribute__((visibility("default"))) rsmi_status_t rsmi_dev_memory_total_get(
    uint32_t dv_ind, rsmi_memory_type_t type, uint64_t* total) {
  rsmi_status_t rc = REAL_RSMI(rsmi_dev_memory_total_get)(dv_ind, type, total);
  if (rc != RSMI_STATUS_SUCCESS || !total || !rsmi_vram(type)) return rc;
  if (uint64_t lim = rsmi_limit(dv_ind)) *total = lim;
  return rc;
}

__attribute__((visibility("default"))) rsmi_status_t rsmi_dev_memory_usage_get(
    uint32_t dv_ind, rsmi_memory_type_t type, uint64_t* used) {
  rsmi_status_t rc = REAL_RSMI(rsmi_dev_memory_usage_get)(dv_ind, type, used);
  if (rc != RSMI_STATUS_SUCCESS || !used || !rsmi_vram(type)) return rc;
  if (uint64_t lim = rsmi_limit(dv_ind)) {
    State& s = st();
    uint64_t u = s.region ? region_device_used(s.region, (int)dv_ind) : 0;
    *used = std::min<uint64_t>(u, lim);
  }
  return rc;
}

// Compute processes on the node (KFD), filtered to this container's own.
__attribute__((visibility("default"))) rsmi_status_t rsmi_compute_process_info_get(
    rsmi_process_info_t* procs, uint32_t* num_items) {
  auto real = REAL_RSMI(rsmi_compute_process_info_get);
  ensure_init();
  if (!st().enabled || !num_items) return real(procs, num_items);
  uint32_t n = 0;
  rsmi_status_t rc = real(nullptr, &n);
  if (rc != RSMI_STATUS_SUCCESS && rc != RSMI_STATUS_INSUFFICIENT_SIZE) return rc;
  std::vector<rsmi_process_info_t> all(n + 16);
  uint32_t got = (uint32_t)all.size();
  rc = real(all.data(), &got);
  if (rc != RSMI_STATUS_SUCCESS && rc != RSMI_STATUS_INSUFFICIENT_SIZE) return rc;
  const std::vector<int> mine = container_host_pids();
  const uint32_t cap = procs ? *num_items : 0;
  uint32_t k = 0;
  for (uint32_t i = 0; i < got && i < all.size(); ++i) {
    if (std::find(mine.begin(), mine.end(), (int)all[i].process_id) == mine.end()) continue;
    if (k < cap) procs[k] = all[i];
    ++k;
  }
  *num_items = k;
  return procs && k > cap ? RSMI_STATUS_INSUFFICIENT_SIZE : RSMI_STATUS_SUCCESS;
}

}  // extern "C"
