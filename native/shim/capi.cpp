// C ABI exported for Python (ctypes): the node monitor attaches to container
// regions through these entry points so every structural write happens under
// the same robust lock the shim uses (the reference monitor writes the mmap
// with no lock at all: cmd/vGPUmonitor/feedback.go:208,231,244).
#include <signal.h>

#include "common.h"
#include "state.h"

using namespace vgpu;

extern "C" {

__attribute__((visibility("default"))) void vgpu_region_layout(vgpu_region_layout_t* out) {
  region_fill_layout(out);
}

__attribute__((visibility("default"))) uint32_t vgpu_region_version() { return VGPU_REGION_VERSION; }

// Create (or attach to and refresh) a region using the limits in the current
// environment.  Returns the mapping or NULL.
__attribute__((visibility("default"))) void* vgpu_region_create(const char* path) {
  DeviceLimits lim = limits_from_env();
  int fd = -1;
  void* r = region_map(path, &lim, &fd);
  if (fd >= 0) close(fd);  // the mapping stays valid after close
  return r;
}

// Attach to an existing, initialised region without modifying it.
__attribute__((visibility("default"))) void* vgpu_region_attach(const char* path) {
  int fd = -1;
  void* r = region_map(path, nullptr, &fd);
  if (fd >= 0) close(fd);
  return r;
}

__attribute__((visibility("default"))) void vgpu_region_detach(void* r) {
  region_unmap((vgpu_shared_region_t*)r, -1);
}

__attribute__((visibility("default"))) int vgpu_region_lock(void* r) {
  return region_lock((vgpu_shared_region_t*)r);
}

__attribute__((visibility("default"))) void vgpu_region_unlock(void* r) {
  region_unlock((vgpu_shared_region_t*)r);
}

__attribute__((visibility("default"))) int vgpu_region_purge(void* r, int host_ns) {
  return region_purge_dead((vgpu_shared_region_t*)r, host_ns != 0);
}

__attribute__((visibility("default"))) int vgpu_region_claim(void* r, int pid, int host_pid, int prio) {
  return region_claim_slot((vgpu_shared_region_t*)r, pid, host_pid, prio);
}

__attribute__((visibility("default"))) void vgpu_region_release(void* r, int slot) {
  region_release_slot((vgpu_shared_region_t*)r, slot);
}

__attribute__((visibility("default"))) uint64_t vgpu_region_device_used(void* r, int dev) {
  return region_device_used((vgpu_shared_region_t*)r, dev);
}

// Feedback words (monitor → shim).  Negative values are left unchanged.
__attribute__((visibility("default"))) void vgpu_region_set_feedback(void* rp, int recent_kernel,
                                                                     int utilization_switch,
                                                                     int set_recent) {
  auto* r = (vgpu_shared_region_t*)rp;
  if (set_recent) __atomic_store_n(&r->recent_kernel, recent_kernel, __ATOMIC_RELAXED);
  if (utilization_switch >= 0)
    __atomic_store_n(&r->utilization_switch, utilization_switch, __ATOMIC_RELAXED);
  __atomic_fetch_add(&r->monitor_seq, 1, __ATOMIC_RELAXED);
}

// Decrement recent_kernel if positive; returns the new value.
__attribute__((visibility("default"))) int vgpu_region_decay_recent(void* rp) {
  auto* r = (vgpu_shared_region_t*)rp;
  int cur = __atomic_load_n(&r->recent_kernel, __ATOMIC_RELAXED);
  while (cur > 0 && !__atomic_compare_exchange_n(&r->recent_kernel, &cur, cur - 1, true,
                                                  __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
  }
  return cur > 0 ? cur - 1 : cur;
}

// Elastic CU resizing: install a new mask for `dev` (words little-endian).
__attribute__((visibility("default"))) int vgpu_region_set_cu_mask(void* rp, int dev,
                                                                   const uint64_t* words) {
  auto* r = (vgpu_shared_region_t*)rp;
  if (dev < 0 || dev >= VGPU_MAX_DEVICES) return -1;
  if (region_lock(r) != 0) return -1;
  for (int w = 0; w < VGPU_CU_MASK_WORDS; ++w)
    __atomic_store_n(&r->dev[dev].cu_mask[w], words[w], __ATOMIC_RELAXED);
  // New plugin generation (after the words: a reader that sees it sees them).
  uint32_t f = __atomic_load_n(&r->dev[dev].flags, __ATOMIC_RELAXED);
  const uint32_t gen = ((f >> VGPU_DEV_POOL_GEN_SHIFT) + 1) & 0xffffu;
  f = (f & ((1u << VGPU_DEV_POOL_GEN_SHIFT) - 1)) | (gen << VGPU_DEV_POOL_GEN_SHIFT);
  __atomic_store_n(&r->dev[dev].flags, f, __ATOMIC_RELEASE);
  region_unlock(r);
  return 0;
}

// Node monitor: record a host pid it resolved for `slot` (src = VGPU_HOSTPID_MONITOR).
// Only a slot that still holds container pid `pid` and is unverified is
// changed, so a slot reused meanwhile is left alone.  Returns 1 if written.
__attribute__((visibility("default"))) int vgpu_region_set_host_pid(void* rp, int slot, int pid, int host_pid,
                                                                    int src) {
  auto* r = (vgpu_shared_region_t*)rp;
  if (slot < 0 || slot >= VGPU_MAX_PROCS || host_pid <= 0) return -1;
  if (region_lock(r) != 0) return -1;
  vgpu_proc_slot_t& s = r->procs[slot];
  int done = 0;
  if (s.status != VGPU_PROC_FREE && s.pid == pid && s.host_pid_src == VGPU_HOSTPID_UNVERIFIED) {
    s.host_pid = host_pid;
    s.host_pid_src = src;
    done = 1;
  }
  region_unlock(r);
  return done;
}

// Signal every live process of the region (suspend_all / resume_all analogue).
__attribute__((visibility("default"))) int vgpu_region_signal_all(void* rp, int sig, int host_ns) {
  auto* r = (vgpu_shared_region_t*)rp;
  int n = 0;
  if (region_lock(r) != 0) return -1;
  for (int i = 0; i < VGPU_MAX_PROCS; ++i) {
    const vgpu_proc_slot_t& s = r->procs[i];
    if (s.status == VGPU_PROC_FREE) continue;
    if (host_ns && s.host_pid_src == VGPU_HOSTPID_UNVERIFIED) continue;
    int pid = host_ns ? s.host_pid : s.pid;
    if (pid > 0 && kill(pid, sig) == 0) ++n;
  }
  region_unlock(r);
  return n;
}

__attribute__((visibility("default"))) uint64_t vgpu_parse_mem(const char* s) { return parse_mem(s); }

__attribute__((visibility("default"))) int vgpu_parse_cu_mask(const char* s, uint64_t* out, int words) {
  return parse_cu_mask(s, out, words);
}

// In-process introspection for tests running under the preload.
__attribute__((visibility("default"))) void* vgpu_self_region() {
  ensure_init();
  return st().region;
}
__attribute__((visibility("default"))) int vgpu_self_slot() {
  ensure_init();
  return st().slot;
}
__attribute__((visibility("default"))) int vgpu_self_enabled() {
  ensure_init();
  return st().enabled ? 1 : 0;
}
__attribute__((visibility("default"))) int vgpu_self_reserve(int dev, uint64_t size) {
  ensure_init();
  return mem_reserve(dev, size, kDeviceBuf) ? 1 : 0;
}
__attribute__((visibility("default"))) void vgpu_self_unreserve(int dev, uint64_t size) {
  mem_unreserve(dev, size, kDeviceBuf);
}
// Pager accounting (vgpu/ops/pager.py): HBM<->host bytes moved by this process.
__attribute__((visibility("default"))) void vgpu_self_add_swap(int dev, uint64_t in_bytes,
                                                               uint64_t out_bytes) {
  ensure_init();
  vgpu_proc_slot_t* sl = my_slot();
  if (!sl || dev < 0 || dev >= VGPU_MAX_DEVICES) return;
  __atomic_fetch_add(&sl->used[dev].swap_in_bytes, in_bytes, __ATOMIC_RELAXED);
  __atomic_fetch_add(&sl->used[dev].swap_out_bytes, out_bytes, __ATOMIC_RELAXED);
}

// Virtual device memory pager counters: bytes promoted / demoted, migrations,
// bytes of spilled ranges now resident in HBM, spilled ranges alive.
__attribute__((visibility("default"))) uint64_t vgpu_self_graph_ranges(hipGraphExec_t exec) {
  return vmem_graph_ranges(exec);
}

__attribute__((visibility("default"))) void vgpu_self_vmem_stats(uint64_t out[5]) {
  ensure_init();
  vmem_stats(&out[0], &out[1], &out[2], &out[3], &out[4]);
}

// Kernel dispatches seen by intercept queues, and how many queues are intercepted
// (hooks_hsa.cpp, HSA_TOOLS_LIB mode).
__attribute__((visibility("default"))) uint64_t vgpu_self_hsa_dispatches() { return g_hsa_dispatches.load(); }
__attribute__((visibility("default"))) int vgpu_self_hsa_intercepted_queues() { return g_hsa_intercepted_queues.load(); }

// VMM suspend vehicle (vmm.cpp): ranges, bytes, evicted bytes, last suspend /
// resume ns, completed suspend-resume cycles, the last suspend's pinning ns and
// the last resume's re-mapping ns.
__attribute__((visibility("default"))) void vgpu_self_vmm_stats(uint64_t out[8]) {
  ensure_init();
  vmm_stats(out);
}

__attribute__((visibility("default"))) void vgpu_self_vmem_budget(int dev, uint64_t out[8]) {
  ensure_init();
  vmem_budget_books(dev, out);
}

__attribute__((visibility("default"))) uint64_t vgpu_self_host_bytes(int dev) {
  ensure_init();
  vgpu_proc_slot_t* sl = my_slot();
  if (!sl || dev < 0 || dev >= VGPU_MAX_DEVICES) return 0;
  return __atomic_load_n(&sl->used[dev].host_bytes, __ATOMIC_RELAXED);
}

// 1 when ROCr handed us its API table (HSA_TOOLS_LIB=libvgpu.so), else 0.
__attribute__((visibility("default"))) int vgpu_self_hsa_table_mode() { return hsa_table_mode() ? 1 : 0; }

// This process's charge on `dev` by class: 0 context/runtime, 1 module, 2 buffer, 3 host, 4 total.
__attribute__((visibility("default"))) uint64_t vgpu_self_usage(int dev, int which) {
  ensure_init();
  vgpu_proc_slot_t* sl = my_slot();
  if (!sl || dev < 0 || dev >= VGPU_MAX_DEVICES) return 0;
  const vgpu_dev_usage_t& u = sl->used[dev];
  const uint64_t* f[] = {&u.context_bytes, &u.module_bytes, &u.buffer_bytes, &u.host_bytes,
                         &u.total_bytes};
  if (which < 0 || which > 4) return 0;
  return __atomic_load_n(f[which], __ATOMIC_RELAXED);
}

// Bytes of other processes' buffers this process has mapped via hipIpcOpenMemHandle.
__attribute__((visibility("default"))) int64_t vgpu_self_ipc_imported(int dev) {
  if (dev < 0 || dev >= VGPU_MAX_DEVICES) return 0;
  return st().ipc_imported[dev].load();
}

// Temporal limiter: fair-share GPU ns charged and wall ns busy on `dev` so far.
__attribute__((visibility("default"))) void vgpu_self_gpu_time(int dev, uint64_t* charged,
                                                               uint64_t* busy) {
  limiter_stats(dev, charged, busy);
}

__attribute__((visibility("default"))) void vgpu_self_share_state(int dev, int64_t out[8]) {
  limiter_share_state(dev, out);
}

__attribute__((visibility("default"))) void vgpu_self_on_launch(int dev, uint64_t wg) {
  ensure_init();
  limiter_on_launch(dev, wg);
}

}  // extern "C"
