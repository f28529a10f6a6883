// Allocation ledger + container-wide HBM cap.
//
// Reference behaviour: lib/nvidia/libvgpu.so allocator.c — allocate_raw →
// add_chunk → oom_check (limit vs Σ shared-region usage, purging exited
// processes via rm_quitted_process) → add_gpu_device_memory_usage; free_raw →
// remove_chunk.  "Device %d OOM %lu / %lu" log line.
//
// Here: the charge is RESERVED in the shared region under the robust lock
// before the real allocator runs (so two processes racing for the last bytes
// cannot both win), and released if the real call fails.
#include <fcntl.h>
#include <signal.h>
#include <unistd.h>

#include "common.h"
#include "state.h"

namespace vgpu {

uint32_t cumask_driver_uid(int dev);  // KFD gpu_id of a device, 0 = unknown

uint64_t mem_limit(int dev) {
  State& s = st();
  if (!s.enabled || dev < 0 || dev >= VGPU_MAX_DEVICES) return 0;
  if (s.region) return s.region->dev[dev].mem_limit;
  return s.lim.mem_limit[dev];
}

uint64_t mem_used(int dev) {
  State& s = st();
  if (!s.region || dev < 0 || dev >= VGPU_MAX_DEVICES) return 0;
  return region_device_used(s.region, dev) + region_device_host_used(s.region, dev);
}

static void add_usage(vgpu_dev_usage_t& u, uint64_t size, int kind, bool add) {
  auto op = [&](uint64_t* f) {
    if (add) __atomic_fetch_add(f, size, __ATOMIC_RELAXED);
    else __atomic_fetch_sub(f, size, __ATOMIC_RELAXED);
  };
  switch (kind) {
    case kIpcImport:
      return;  // another process's buffer: charged to its exporter only
    case kPinnedHost:
      return;  // host memory: pinned_host_bytes (pools.cpp), not the HBM cap
    case kHostSpill:
      op(&u.host_bytes);
      return;
    case kModule:
      op(&u.module_bytes);
      break;
    case kRuntime:
      op(&u.context_bytes);
      break;
    default:
      op(&u.buffer_bytes);
      break;
  }
  op(&u.total_bytes);
}

// High-water mark; called only once an allocation has really succeeded (a
// reservation that the runtime then refuses must not move the peak).
static void note_peak(vgpu_dev_usage_t& u) {
  uint64_t t = __atomic_load_n(&u.total_bytes, __ATOMIC_RELAXED);
  uint64_t pk = __atomic_load_n(&u.peak_bytes, __ATOMIC_RELAXED);
  while (t > pk && !__atomic_compare_exchange_n(&u.peak_bytes, &pk, t, true, __ATOMIC_RELAXED,
                                                __ATOMIC_RELAXED)) {
  }
}

static bool mem_reserve_once(int dev, uint64_t size, int kind, bool quiet);

// Reserve `size` against the container's cap.  Before refusing, memory that
// stream-ordered pools hold for reuse is trimmed and re-read (pools.cpp).
bool mem_reserve(int dev, uint64_t size, int kind) {
  if (mem_limit(dev)) mem_sync_runtime(dev);
  if (mem_reserve_once(dev, size, kind, true)) return true;
  if (pools_any()) {
    pools_sync(true);
    if (mem_reserve_once(dev, size, kind, true)) return true;
  }
  return mem_reserve_once(dev, size, kind, false);
}

static bool mem_reserve_once(int dev, uint64_t size, int kind, bool quiet) {
  State& s = st();
  vgpu_proc_slot_t* sl = my_slot();
  if (!s.enabled || !sl || dev < 0 || dev >= VGPU_MAX_DEVICES) return true;
  uint64_t limit = s.region->dev[dev].mem_limit;
  if (limit == 0) {  // unlimited: account only
    add_usage(sl->used[dev], size, kind, true);
    return true;
  }
  if (region_lock(s.region) != 0) return true;
  uint64_t used = region_device_used(s.region, dev) + region_device_host_used(s.region, dev);
  if (used + size > limit) {
    region_purge_dead_locked(s.region, false);
    used = region_device_used(s.region, dev) + region_device_host_used(s.region, dev);
  }
  bool ok = used + size <= limit;
  if (ok) add_usage(sl->used[dev], size, kind, true);
  else if (!quiet) __atomic_fetch_add(&sl->oom_events, 1, __ATOMIC_RELAXED);
  region_unlock(s.region);
  if (!ok && !quiet) {
    trace_emit(VGPU_EV_OOM, dev, size, limit);
    VLOG_WARN("Device %d OOM %llu / %llu (request %llu bytes)", dev,
              (unsigned long long)(used + size), (unsigned long long)limit,
              (unsigned long long)size);
    if (s.active_oom_killer) {
      VLOG_ERR("ACTIVE_OOM_KILLER: terminating pid %d", s.pid);
      kill(s.pid, SIGKILL);
    }
  }
  return ok;
}

void mem_unreserve(int dev, uint64_t size, int kind) {
  State& s = st();
  vgpu_proc_slot_t* sl = my_slot();
  if (!s.enabled || !sl || dev < 0 || dev >= VGPU_MAX_DEVICES) return;
  add_usage(sl->used[dev], size, kind, false);
}

void ipc_import_account(int dev, int64_t delta) {
  if (dev < 0 || dev >= VGPU_MAX_DEVICES) return;
  st().ipc_imported[dev].fetch_add(delta, std::memory_order_relaxed);
}

std::atomic<int64_t> g_app_managed{0};  // live hipMallocManaged allocations of the application

bool app_has_managed() { return g_app_managed.load(std::memory_order_relaxed) > 0; }

void ledger_add(void* p, uint64_t size, int dev, int kind) {
  State& s = st();
  trace_emit(VGPU_EV_ALLOC, dev, size, (uint64_t)kind);
  {
    std::lock_guard<std::mutex> g(s.ledger_mu);
    s.ledger[(uintptr_t)p] = Alloc{size, dev, kind};
  }
  if (kind == kManaged) g_app_managed.fetch_add(1, std::memory_order_relaxed);
  vgpu_proc_slot_t* sl = my_slot();
  if (sl && dev >= 0 && dev < VGPU_MAX_DEVICES) note_peak(sl->used[dev]);
}

bool ledger_take_if(void* p, int kind, Alloc* out) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.ledger_mu);
  auto it = s.ledger.find((uintptr_t)p);
  if (it == s.ledger.end() || it->second.kind != kind) return false;
  *out = it->second;
  s.ledger.erase(it);
  if (out->kind == kManaged) g_app_managed.fetch_sub(1, std::memory_order_relaxed);
  trace_emit(VGPU_EV_FREE, out->dev, out->size, (uint64_t)out->kind);
  return true;
}

void mem_charge_nofail(int dev, uint64_t size, int kind) {
  State& s = st();
  vgpu_proc_slot_t* sl = my_slot();
  if (!s.enabled || !sl || dev < 0 || dev >= VGPU_MAX_DEVICES) return;
  add_usage(sl->used[dev], size, kind, true);
}

bool ledger_take(void* p, Alloc* out) {
  State& s = st();
  {
    std::lock_guard<std::mutex> g(s.ledger_mu);
    auto it = s.ledger.find((uintptr_t)p);
    // An IPC mapping is released only by hipIpcCloseMemHandle (ledger_take_if).
    if (it == s.ledger.end() || it->second.kind == kIpcImport) return false;
    *out = it->second;
    s.ledger.erase(it);
  }
  if (out->kind == kManaged) g_app_managed.fetch_sub(1, std::memory_order_relaxed);
  trace_emit(VGPU_EV_FREE, out->dev, out->size, (uint64_t)out->kind);
  return true;
}

void charge_context(int dev) {
  State& s = st();
  if (!s.enabled || dev < 0 || dev >= VGPU_MAX_DEVICES) return;
  int expected = 0;
  if (!s.dev_touched[dev].compare_exchange_strong(expected, 1)) return;
  vgpu_proc_slot_t* sl = my_slot();
  if (!sl || s.context_charge == 0) return;
  std::lock_guard<std::mutex> g(s.ctx_mu);
  __atomic_fetch_add(&sl->used[dev].context_bytes, s.context_charge, __ATOMIC_RELAXED);
  __atomic_fetch_add(&sl->used[dev].total_bytes, s.context_charge, __ATOMIC_RELAXED);
  s.ctx_booked[dev] += s.context_charge;
}

// The runtime's own VRAM is invisible to the allocation hooks: every hardware
// queue carries a context-save area sized for all 256 CUs (~0.5 GB per queue on
// MI355X, measured: scripts/pool_kfd_probe.py), the stream-ordered pools' VM
// heap keeps physical slack, code objects and scratch live in VRAM.  The
// reference books a fixed context size; here KFD's per-process counter
// (/sys/class/kfd/kfd/proc/<host pid>/vram_<gpu id>, updated as buffer objects
// are created and destroyed) minus the ledger's charge IS that overhead.  It is
// booked as context bytes, between VGPU_CONTEXT_CHARGE and VGPU_CONTEXT_MAX
// (the upper bound guards against counters that also hold imported buffers).
static int kfd_vram_fd(int dev) {
  State& s = st();
  int fd = s.kfd_vram_fd[dev].load(std::memory_order_acquire);
  if (fd != -2) return fd;
  // Not there yet (host pid unresolved, no KFD entry): look again at most every 100 ms.
  static std::atomic<uint64_t> next_try[VGPU_MAX_DEVICES];
  const uint64_t now = mono_ns();
  if (now < next_try[dev].load(std::memory_order_relaxed)) return -1;
  next_try[dev].store(now + 100000000ull, std::memory_order_relaxed);
  int src = 0;
  int pid = self_host_pid(&src);
  if (src == VGPU_HOSTPID_UNVERIFIED) {
    vgpu_proc_slot_t* sl = my_slot();
    if (!sl || __atomic_load_n(&sl->host_pid_src, __ATOMIC_ACQUIRE) == VGPU_HOSTPID_UNVERIFIED)
      return -1;  // not known yet: try again later
    pid = __atomic_load_n(&sl->host_pid, __ATOMIC_RELAXED);
  }
  const uint32_t uid = cumask_driver_uid(dev);
  if (pid <= 0 || !uid) return -1;
  char path[512];
  snprintf(path, sizeof path, "%s/%d/vram_%u", kfd_proc_dir(), pid, uid);
  fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -1;
  int expected = -2;
  if (!s.kfd_vram_fd[dev].compare_exchange_strong(expected, fd)) {
    if (fd >= 0) close(fd);
    return expected;
  }
  VLOG_DEBUG("device %d: runtime VRAM measured from %s", dev, path);
  return fd;
}

void mem_sync_runtime(int dev) {
  State& s = st();
  vgpu_proc_slot_t* sl = my_slot();
  if (!s.enabled || !sl || !s.ctx_measure || dev < 0 || dev >= VGPU_MAX_DEVICES) return;
  if (!s.dev_touched[dev].load(std::memory_order_relaxed)) return;
  const int fd = kfd_vram_fd(dev);
  if (fd < 0) return;
  char buf[32];
  const ssize_t n = pread(fd, buf, sizeof buf - 1, 0);
  if (n <= 0) return;
  buf[n] = 0;
  uint64_t kfd = strtoull(buf, nullptr, 10);
  // KFD's per-process counter includes buffers mapped from other processes
  // (IPC imports: DDP peers, torch CUDA-IPC tensors); their exporters hold
  // the charge (hooks_array.cpp), so they are not this process's context.
  const int64_t imported = s.ipc_imported[dev].load(std::memory_order_relaxed);
  if (imported > 0) kfd = kfd > (uint64_t)imported ? kfd - (uint64_t)imported : 0;
  std::lock_guard<std::mutex> g(s.ctx_mu);
  uint64_t& booked = s.ctx_booked[dev];
  const uint64_t total = __atomic_load_n(&sl->used[dev].total_bytes, __ATOMIC_RELAXED);
  const uint64_t seen = total > booked ? total - booked : 0;
  uint64_t want = kfd > seen ? kfd - seen : 0;
  want = std::min(std::max(want, s.context_charge), std::max(s.ctx_max, s.context_charge));
  if (want == booked) return;
  if (want > booked) {
    __atomic_fetch_add(&sl->used[dev].context_bytes, want - booked, __ATOMIC_RELAXED);
    __atomic_fetch_add(&sl->used[dev].total_bytes, want - booked, __ATOMIC_RELAXED);
  } else {
    __atomic_fetch_sub(&sl->used[dev].context_bytes, booked - want, __ATOMIC_RELAXED);
    __atomic_fetch_sub(&sl->used[dev].total_bytes, booked - want, __ATOMIC_RELAXED);
  }
  booked = want;
}

void mem_after_fork() {
  State& s = st();
  new (&s.ctx_mu) std::mutex();
  for (int d = 0; d < VGPU_MAX_DEVICES; ++d) {
    s.ctx_booked[d] = 0;
    const int fd = s.kfd_vram_fd[d].exchange(-2);
    if (fd >= 0) close(fd);
  }
}

}  // namespace vgpu
