// Stream-ordered memory pools, graph memory and page-locked host memory.
//
// Reference: lib/nvidia/libvgpu.so hooks cuMemAllocAsync, cuMemAllocFromPoolAsync
// (SURVEY.md §2.6 E1b), cuMemHostAlloc (715 B) and cuMemAllocHost_v2 (697 B).
//
// A stream-ordered pool keeps the physical memory of freed blocks for reuse
// (and, with a high release threshold, for good), and a graph's memory-alloc
// nodes draw from the device's graph pool when the graph is LAUNCHED, not when
// it is captured.  Charging hipMallocAsync's `size` at the call and releasing it
// at hipFreeAsync would therefore let physical use drift past the cap
// (VERDICT r2, weak 7).  Here the charge of a pool IS its reserved size:
//   * hipMallocAsync / hipMallocFromPoolAsync reserve `size` against the cap
//     tentatively, allocate, then replace the tentative charge by the growth of
//     the pool's hipMemPoolAttrReservedMemCurrent (a reused block costs 0);
//   * freed blocks stay charged while the pool holds them; before anything is
//     refused for lack of room every pool is trimmed (hipMemPoolTrimTo) and
//     re-read, and the limiter thread re-reads them every 50 ms;
//   * launches captured into a graph are not charged at capture; an executable
//     graph's alloc nodes (the peak of bytes live at once between the captured
//     hipMallocAsync / hipFreeAsync calls) are checked against the cap before
//     each hipGraphLaunch, and the device's graph pool
//     (hipGraphMemAttrReservedMemCurrent) is charged after it.
// Page-locked host memory is booked per process (pinned_host_bytes) and refused
// past VGPU_PINNED_HOST_LIMIT (MiB, container-wide) when set.
#include <algorithm>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "common.h"
#include "real.h"
#include "state.h"

namespace vgpu {

namespace {

struct PoolCharge {
  int dev = -1;
  uint64_t charged = 0;  // bytes of this pool currently booked against the cap
};

std::mutex g_pmu;
std::unordered_map<const void*, PoolCharge> g_pools;  // hipMemPool_t -> charge
uint64_t g_graph_charged[VGPU_MAX_DEVICES] = {};      // device graph pool charge
// Graph alloc nodes: the peak of bytes live at once among a capture's
// hipMallocAsync / hipFreeAsync pairs (a graph's free nodes let the graph pool
// reuse memory inside one launch), per capture id, then per graph, then per
// executable.
struct CapMem {
  uint64_t live = 0, peak = 0;
};
std::unordered_map<unsigned long long, CapMem> g_cap_mem;
std::unordered_map<const void*, std::pair<unsigned long long, uint64_t>> g_cap_ptrs;  // ptr -> (cid, size)
std::unordered_map<const void*, uint64_t> g_graph_bytes, g_exec_bytes;

uint64_t pool_reserved(hipMemPool_t pool) {
  auto get = REAL_HIP(hipMemPoolGetAttribute);
  uint64_t v = 0;
  if (!get || get(pool, hipMemPoolAttrReservedMemCurrent, &v) != hipSuccess) return UINT64_MAX;
  return v;
}

uint64_t graph_reserved(int dev) {
  auto get = REAL_HIP(hipDeviceGetGraphMemAttribute);
  uint64_t v = 0;
  if (!get || get(dev, hipGraphMemAttrReservedMemCurrent, &v) != hipSuccess) return UINT64_MAX;
  return v;
}

// Book `now` as the charge that was `was` (caller holds g_pmu).
void rebook(int dev, uint64_t& was, uint64_t now) {
  if (now == UINT64_MAX || now == was) return;
  if (now > was) mem_charge_nofail(dev, now - was, kDeviceBuf);
  else mem_unreserve(dev, was - now, kDeviceBuf);
  was = now;
}

void sync_pool_locked(hipMemPool_t pool, PoolCharge& c) { rebook(c.dev, c.charged, pool_reserved(pool)); }

unsigned long long capture_of(hipStream_t stream) {
  if (g_open_captures.load(std::memory_order_acquire) == 0) return 0;
  auto info = REAL_HIP(hipStreamGetCaptureInfo);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  if (!info || info(stream, &cs, &id) != hipSuccess || cs != hipStreamCaptureStatusActive) return 0;
  return id ? id : 1;
}

}  // namespace

// Re-read every pool's reserved size (and trim first when `trim`): the limiter
// thread calls it periodically, mem_reserve before it refuses an allocation.
void pools_sync(bool trim) {
  std::lock_guard<std::mutex> l(g_pmu);
  for (auto& kv : g_pools) {
    auto pool = (hipMemPool_t)kv.first;
    if (trim) (void)REAL_HIP(hipMemPoolTrimTo)(pool, 0);
    sync_pool_locked(pool, kv.second);
  }
  for (int d = 0; d < VGPU_MAX_DEVICES; ++d) {
    if (!g_graph_charged[d]) continue;
    if (trim) (void)REAL_HIP(hipDeviceGraphMemTrim)(d);
    rebook(d, g_graph_charged[d], graph_reserved(d));
  }
  (void)REAL_HIP(hipGetLastError)();
}

bool pools_any() {
  std::lock_guard<std::mutex> l(g_pmu);
  return !g_pools.empty() || [] {
    for (uint64_t c : g_graph_charged)
      if (c) return true;
    return false;
  }();
}

hipError_t pool_alloc_async(void** ptr, size_t size, hipStream_t stream, hipMemPool_t pool,
                            hipError_t (*real)(void**, size_t, hipMemPool_t, hipStream_t, bool)) {
  ensure_init();
  State& s = st();
  const bool from_pool = pool != nullptr;
  if (!s.enabled || size == 0) return real(ptr, size, pool, stream, from_pool);
  const int dev = tl_device;
  if (const unsigned long long cid = capture_of(stream)) {
    // A graph memory-alloc node: physical memory comes from the graph pool
    // when the graph runs; account it at hipGraphLaunch.
    hipError_t rc = real(ptr, size, pool, stream, from_pool);
    if (rc == hipSuccess) {
      std::lock_guard<std::mutex> l(g_pmu);
      CapMem& m = g_cap_mem[cid];
      m.live += size;
      m.peak = std::max(m.peak, m.live);
      g_cap_ptrs[*ptr] = {cid, (uint64_t)size};
    }
    return rc;
  }
  suspend_gate();
  charge_context(dev);
  if (!pool && REAL_HIP(hipDeviceGetMemPool)(&pool, dev) != hipSuccess) {
    (void)REAL_HIP(hipGetLastError)();
    pool = nullptr;
  }
  if (!mem_reserve(dev, size, kDeviceBuf)) {
    // Freed blocks the pool still holds are charged: give them back and retry.
    (void)REAL_HIP(hipStreamSynchronize)(stream);
    pools_sync(true);
    if (!mem_reserve(dev, size, kDeviceBuf)) return hipErrorOutOfMemory;
  }
  hipError_t rc = real(ptr, size, pool, stream, from_pool);
  VLOG_DEBUG("stream-ordered alloc %zu bytes (pool %p, stream %p, device %d) -> %d", size, (void*)pool,
             (void*)stream, dev, (int)rc);
  if (rc == hipSuccess && pool) {
    std::lock_guard<std::mutex> l(g_pmu);
    PoolCharge& c = g_pools[(const void*)pool];
    c.dev = dev;
    sync_pool_locked(pool, c);  // the pool's growth (0 when a freed block was reused)
  }
  if (rc != hipSuccess || pool) mem_unreserve(dev, size, kDeviceBuf);  // tentative charge -> pool charge
  if (rc == hipSuccess && !pool) ledger_add(*ptr, size, dev, kDeviceBuf);  // no pool to read: plain charge
  return rc;
}

// ---- graphs -------------------------------------------------------------------------------
// hipFreeAsync of a block a capture allocated: a free node of that capture.
void pools_capture_free(const void* ptr) {
  if (!ptr) return;
  std::lock_guard<std::mutex> l(g_pmu);
  auto it = g_cap_ptrs.find(ptr);
  if (it == g_cap_ptrs.end()) return;
  auto m = g_cap_mem.find(it->second.first);
  if (m != g_cap_mem.end()) m->second.live -= std::min(m->second.live, it->second.second);
  g_cap_ptrs.erase(it);
}

void pools_capture_ended(unsigned long long cid, hipGraph_t graph) {
  std::lock_guard<std::mutex> l(g_pmu);
  for (auto it = g_cap_ptrs.begin(); it != g_cap_ptrs.end();)
    it = it->second.first == cid ? g_cap_ptrs.erase(it) : std::next(it);
  auto it = g_cap_mem.find(cid);
  if (it == g_cap_mem.end()) return;
  if (graph) g_graph_bytes[graph] += it->second.peak;
  g_cap_mem.erase(it);
}

// hipGraphAddMemAllocNode: the node's bytes are charged at launch like a
// captured hipMallocAsync's.  Free nodes are not netted out (an upper bound:
// the graph pool may reuse a freed block inside one launch).
void pools_graph_add_bytes(hipGraph_t graph, uint64_t bytes) {
  if (!graph || !bytes) return;
  std::lock_guard<std::mutex> l(g_pmu);
  g_graph_bytes[graph] += bytes;
}

void pools_graph_child(hipGraph_t graph, hipGraph_t child) {
  std::lock_guard<std::mutex> l(g_pmu);
  auto it = g_graph_bytes.find(child);
  if (it != g_graph_bytes.end() && it->second) {
    const uint64_t b = it->second;
    g_graph_bytes[graph] += b;
  }
}

void pools_graph_instantiated(hipGraph_t graph, hipGraphExec_t exec) {
  std::lock_guard<std::mutex> l(g_pmu);
  auto it = g_graph_bytes.find(graph);
  if (it == g_graph_bytes.end()) g_exec_bytes.erase(exec);
  else g_exec_bytes[exec] = it->second;
}

void pools_graph_destroyed(const void* graph_or_exec) {
  std::lock_guard<std::mutex> l(g_pmu);
  g_graph_bytes.erase(graph_or_exec);
  g_exec_bytes.erase(graph_or_exec);
}

uint64_t pools_exec_bytes(hipGraphExec_t exec) {
  std::lock_guard<std::mutex> l(g_pmu);
  auto it = g_exec_bytes.find(exec);
  return it == g_exec_bytes.end() ? 0 : it->second;
}

// Before a launch: can the graph pool grow to hold this graph's alloc nodes?
// Reserves the possible growth tentatively; *tentative receives it.
bool pools_graph_admit(hipGraphExec_t exec, int dev, uint64_t* tentative) {
  *tentative = 0;
  if (!st().enabled || dev < 0 || dev >= VGPU_MAX_DEVICES) return true;
  const uint64_t need = pools_exec_bytes(exec);
  if (!need) return true;
  auto growth = [&] {
    std::lock_guard<std::mutex> l(g_pmu);
    return need > g_graph_charged[dev] ? need - g_graph_charged[dev] : 0;
  };
  // mem_reserve may trim the pools (graph pool included) before it succeeds,
  // which raises the growth this launch needs: re-check after every reserve.
  for (int tries = 0; tries < 3; ++tries) {
    const uint64_t grow = growth();
    if (!grow) return true;
    if (!mem_reserve(dev, grow, kDeviceBuf)) return false;
    if (growth() <= grow) {
      *tentative = grow;
      return true;
    }
    mem_unreserve(dev, grow, kDeviceBuf);
  }
  return false;
}

void pools_graph_launched(int dev, uint64_t tentative) {
  if (dev < 0 || dev >= VGPU_MAX_DEVICES) return;
  {
    std::lock_guard<std::mutex> l(g_pmu);
    const uint64_t r = graph_reserved(dev);
    if (r != UINT64_MAX && (r || g_graph_charged[dev])) rebook(dev, g_graph_charged[dev], r);
  }
  if (tentative) mem_unreserve(dev, tentative, kDeviceBuf);
}

// ---- page-locked host memory --------------------------------------------------------------
bool pinned_reserve(uint64_t size) {
  State& s = st();
  vgpu_proc_slot_t* sl = my_slot();
  if (!s.enabled || !sl) return true;
  static const uint64_t limit = parse_mem(env_first("VGPU_PINNED_HOST_LIMIT"));
  if (limit && region_lock(s.region) == 0) {
    uint64_t used = 0;
    for (int i = 0; i < VGPU_MAX_PROCS; ++i)
      if (s.region->procs[i].status != VGPU_PROC_FREE) used += s.region->procs[i].pinned_host_bytes;
    const bool ok = used + size <= limit;
    if (ok) __atomic_fetch_add(&sl->pinned_host_bytes, size, __ATOMIC_RELAXED);
    region_unlock(s.region);
    if (!ok)
      VLOG_WARN("pinned host memory %llu / %llu (request %llu bytes) refused", (unsigned long long)used,
                (unsigned long long)limit, (unsigned long long)size);
    return ok;
  }
  __atomic_fetch_add(&sl->pinned_host_bytes, size, __ATOMIC_RELAXED);
  return true;
}

void pinned_release(uint64_t size) {
  if (vgpu_proc_slot_t* sl = my_slot()) __atomic_fetch_sub(&sl->pinned_host_bytes, size, __ATOMIC_RELAXED);
}

void pools_after_fork() {
  new (&g_pmu) std::mutex();
  g_pools.clear();
  for (auto& c : g_graph_charged) c = 0;
  g_cap_mem.clear();
  g_cap_ptrs.clear();
  g_graph_bytes.clear();
  g_exec_bytes.clear();
}

}  // namespace vgpu
