// Transparent virtual device memory (VGPU_OVERSUBSCRIBE=true).
//
// Reference: the NVIDIA libvgpu.so backs an oversubscribed pod with
// cuMemAllocManaged (README.md:283-287,
// pkg/device-plugin/nvidiadevice/nvinternal/plugin/server.go:348-350) and
// leaves page migration to the UVM driver's fault handler.  MI355X runs with
// XNACK off, so there are no recoverable GPU page faults: nothing migrates
// unless somebody asks.  This module is that somebody.
//
// Measured on MI355X (native/probes/svm_probe.hip, profiles/vmem_r2.md):
// host-located VMM handles are refused (hipMemCreate -> invalid value), so a
// VA-stable HBM <-> host swap has exactly one vehicle, a KFD SVM range
// (hipMallocManaged).  The GPU reads one in place from host memory at the
// zero-copy rate (55 GB/s) and at HBM speed (5.3 TB/s) once it lives in
// VRAM; hsa_amd_svm_prefetch_async moves it at ~6 GB/s up / ~10 GB/s down
// (hipMemPrefetchAsync goes through a slower path: 1.3-2 GB/s), with the
// process's queues paused by KFD during the move, so it is always safe.
//
// Design:
//   * every pod has a physical HBM budget per device (region dev[].mem_physical,
//     VGPU_DEVICE_MEMORY_PHYSICAL_<i>; the device plugin sets cap / memory
//     scaling on an oversubscribed node, so co-located pods split the HBM
//     instead of the first one to allocate taking it all).  0 = whole device;
//   * with a budget, every device allocation of at least VGPU_VMEM_MANAGED_MIN_MB
//     (32) is a coarse-grained managed range from the start, made resident at
//     once while the budget (and physical HBM beyond the headroom) has room,
//     after demoting cold ranges -- so memory a pod no longer uses can give way
//     to memory it does (a second model, an idle KV pool).  Without a budget,
//     only an allocation that no longer fits in physical HBM becomes a
//     managed range (it starts host-resident);
//   * every kernel launch scans its argument blob for pointers into those
//     ranges (the HIP-Clang stub's argument array lives in the caller's
//     frame; module launches carry a sized kernarg buffer) and stamps the
//     range's last-use tick — no metadata, no device-side cost, and a missed
//     or spurious hit only costs performance, never correctness;
//   * launches captured into a hipGraph are scanned the same way at capture
//     time and the ranges they name are kept per capture -> graph -> exec;
//     every hipGraphLaunch stamps them (a replayed graph runs no hooks);
//   * a pager thread promotes recently used host-resident ranges into HBM
//     while the budget and physical HBM have room, and demotes ranges that
//     went cold when a hotter one is waiting or a new allocation needs the
//     room.  Hot ranges are never demoted for other hot ranges: when the hot
//     set exceeds the budget the resident part stays put and the rest is read
//     in place (zero-copy), which for a cyclic sweep beats any LRU exchange;
//   * SIGUSR2 (suspend) demotes everything the process holds in HBM through
//     managed ranges; after SIGUSR1 ranges come back as they are used;
//   * charges never change (the cap counts HBM + host), only where they are
//     booked: host_bytes <-> buffer/total bytes, plus swap_in/swap_out bytes
//     and VGPU_EV_MIGRATE trace events.
// KFD moves SVM pages at 6-7 GB/s up and 9-11 GB/s down on MI355X regardless
// of piece size, transparent huge pages or concurrency (native/probes/
// svm_rate.hip, profiles/vmem_r3.md), so the pager moves whole ranges in
// 1 GiB pieces and never cycles; the last piece that fits is cut to the
// budget's remaining room, after the plain buffers' recent high-water mark
// (plain_reserve: activations are placed ahead of weights).
// VGPU_VMEM_MIGRATE=0 keeps the round-1 behaviour (pinned zero-copy spill).
#include <pthread.h>
#include <sys/mman.h>

#include <new>

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <string>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <shared_mutex>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "common.h"
#include "real.h"
#include "state.h"

namespace vgpu {

namespace {

struct VRange {
  uintptr_t base;
  uint64_t size;
  int dev;
  uint64_t gpu_bytes;                      // promoted prefix [base, base + gpu_bytes)
  std::atomic<uint64_t> last_use{0};       // pager tick of the latest launch that named it
  std::atomic<uint32_t> uses{0};           // launches that named it (halved every second)
  bool pager_owned_gpu = false;            // promoted by the pager (so it may demote it)
  VRange(uintptr_t b, uint64_t s, int d) : base(b), size(s), dev(d), gpu_bytes(0) {}
};

std::shared_mutex g_tab_mu;                // guards g_tab's shape (launch hooks take it shared)
std::vector<VRange*> g_tab;                // sorted by base
std::atomic<int> g_count{0};
std::mutex g_move_mu;                      // one migration or free at a time
std::atomic<uint64_t> g_tick{1};
std::atomic<uint64_t> g_in_bytes{0}, g_out_bytes{0}, g_moves{0};

std::mutex g_thr_mu;
std::condition_variable g_thr_cv;
bool g_thr_run = false;          // guarded by g_thr_mu
std::atomic<int> g_thr_alive{0};

struct Knobs {
  bool on = true;
  uint64_t headroom = 2ull << 30;
  int tick_ms = 50;
  uint64_t hot_ticks = 20;   // used within the last second -> promote
  uint64_t cold_ticks = 40;  // unused for two seconds -> may be demoted
  uint64_t piece = 1ull << 30;
  int64_t managed_min = 32ll << 20;  // with a physical budget: allocations this large are managed ranges
  // VGPU_SUSPEND_EVICT (device plugin --suspend-evict): managed ranges without a
  // budget or oversubscription, resident like hipMalloc memory, so a suspend
  // (SIGUSR2) can give the container's HBM back.
  bool suspend_evict = false;
  uint64_t plain_window_ms = 30000;  // plain high-water mark window (plain_reserve)
  bool cut_pieces = true;            // VGPU_VMEM_CUT_PIECES=0: whole pieces only (A/B)
  // madvise(MADV_HUGEPAGE) on managed ranges: their host-resident pages are read
  // over the host link in 2 MiB pages (part E at equal HBM: 6.9-7.3 -> 7.5 tok/s,
  // zero-copy 7.8; profiles/r4/vmem/part_e_context_charge*.log).  VGPU_VMEM_THP=0: off.
  bool thp = true;
  // A graph launch whose ranges are mostly on the host waits (at most this
  // long) for the pager to bring them in — a model switch (vmem_graph_launched).
  uint64_t gate_ms = 10000;
};

const Knobs& knobs() {
  static Knobs k = [] {
    Knobs v;
    v.on = env_bool(env_first("VGPU_VMEM_MIGRATE"), true);
    if (const char* e = env_first("VGPU_VMEM_HEADROOM_MB")) v.headroom = strtoull(e, nullptr, 10) << 20;
    if (const char* e = env_first("VGPU_VMEM_TICK_MS")) v.tick_ms = std::max(1, atoi(e));
    if (const char* e = env_first("VGPU_VMEM_HOT_MS")) v.hot_ticks = std::max<uint64_t>(1, strtoull(e, nullptr, 10) / v.tick_ms);
    if (const char* e = env_first("VGPU_VMEM_COLD_MS"))
      v.cold_ticks = std::max<uint64_t>(1, strtoull(e, nullptr, 10) / v.tick_ms);
    if (const char* e = env_first("VGPU_VMEM_PIECE_MB")) v.piece = std::max<uint64_t>(2, strtoull(e, nullptr, 10)) << 20;
    v.suspend_evict = env_bool(env_first("VGPU_SUSPEND_EVICT"), false);
    if (const char* e = env_first("VGPU_VMEM_PLAIN_WINDOW_MS")) v.plain_window_ms = std::max(1ull, strtoull(e, nullptr, 10));
    v.cut_pieces = env_bool(env_first("VGPU_VMEM_CUT_PIECES"), true);
    v.thp = env_bool(env_first("VGPU_VMEM_THP"), true);
    if (const char* e = env_first("VGPU_VMEM_GATE_MS")) v.gate_ms = strtoull(e, nullptr, 10);
    if (const char* e = env_first("VGPU_VMEM_MANAGED_MIN_MB")) {
      const long long mb = atoll(e);
      v.managed_min = mb < 0 ? -1 : (int64_t)mb << 20;
    }
    return v;
  }();
  return k;
}

VRange* find_locked(uintptr_t p) {
  auto it = std::upper_bound(g_tab.begin(), g_tab.end(), p, [](uintptr_t v, const VRange* r) { return v < r->base; });
  if (it == g_tab.begin()) return nullptr;
  VRange* r = *(it - 1);
  return p < r->base + r->size ? r : nullptr;
}

// Ranges named by launches of the calling thread while its stream is being
// captured (vmem_scan_*): they belong to the graph, not to this instant.
thread_local std::vector<uintptr_t>* tl_sink = nullptr;
// Set while the arguments of an explicitly built graph node are read: the
// ranges go to tl_sink only (nothing runs now, so nothing is stamped as used).
thread_local bool tl_collect_only = false;
std::atomic<int> g_wake{0};  // a launch named a range that is not fully in HBM
// Tick at which a gated graph launch (vmem_graph_launched) started waiting, 0
// when none: ranges unused since then may give way at once.
std::atomic<uint64_t> g_gate_tick{0};
std::mutex g_nogate_mu;
std::unordered_set<const void*> g_nogate;  // executables whose gate gave up (they do not fit)

inline void touch_word(uintptr_t w, uint64_t tick) {
  if (w < g_tab.front()->base || w >= g_tab.back()->base + g_tab.back()->size) return;
  if (tl_collect_only) {
    if (VRange* r = find_locked(w))
      if (tl_sink) tl_sink->push_back(r->base);
    return;
  }
  if (VRange* r = find_locked(w)) {
    if (r->last_use.load(std::memory_order_relaxed) != tick) r->last_use.store(tick, std::memory_order_relaxed);
    r->uses.fetch_add(1, std::memory_order_relaxed);
    if (r->gpu_bytes < r->size && !g_wake.load(std::memory_order_relaxed)) g_wake.store(1, std::memory_order_relaxed);
    if (tl_sink) tl_sink->push_back(r->base);
  }
}

void scan_words_locked(const unsigned char* p, size_t n, uint64_t tick) {
  for (size_t off = 0; off + sizeof(uintptr_t) <= n; off += 4) {  // kernargs are 4-byte aligned at least
    uintptr_t w;
    memcpy(&w, p + off, sizeof w);
    touch_word(w, tick);
  }
}

// Bounds of the calling thread's stack: [frame of the scanner, top of stack).
uintptr_t stack_top() {
  static thread_local uintptr_t top = 0;
  if (!top) {
    pthread_attr_t a;
    void* lo = nullptr;
    size_t sz = 0;
    if (pthread_getattr_np(pthread_self(), &a) == 0) {
      pthread_attr_getstack(&a, &lo, &sz);
      pthread_attr_destroy(&a);
    }
    top = lo ? (uintptr_t)lo + sz : 1;
  }
  return top;
}

// ---- accounting ----------------------------------------------------------------------
void book_move(int dev, uint64_t bytes, bool to_gpu) {
  vgpu_proc_slot_t* sl = my_slot();
  if (!sl || dev < 0 || dev >= VGPU_MAX_DEVICES || !bytes) return;
  vgpu_dev_usage_t& u = sl->used[dev];
  if (to_gpu) {
    __atomic_fetch_sub(&u.host_bytes, bytes, __ATOMIC_RELAXED);
    __atomic_fetch_add(&u.buffer_bytes, bytes, __ATOMIC_RELAXED);
    __atomic_fetch_add(&u.total_bytes, bytes, __ATOMIC_RELAXED);
    __atomic_fetch_add(&u.swap_in_bytes, bytes, __ATOMIC_RELAXED);
  } else {
    __atomic_fetch_sub(&u.buffer_bytes, bytes, __ATOMIC_RELAXED);
    __atomic_fetch_sub(&u.total_bytes, bytes, __ATOMIC_RELAXED);
    __atomic_fetch_add(&u.host_bytes, bytes, __ATOMIC_RELAXED);
    __atomic_fetch_add(&u.swap_out_bytes, bytes, __ATOMIC_RELAXED);
  }
}

// ---- migration --------------------------------------------------------------------------
bool prefetch(uintptr_t p, uint64_t n, int dev, bool to_gpu) {
  hsa_agent_t agent;
  if (!(to_gpu ? hsa_gpu_agent(dev, &agent) : hsa_cpu_agent(&agent))) return false;
  hsa_signal_t sig;
  if (REAL_HSA(hsa_signal_create)(1, 0, nullptr, &sig) != HSA_STATUS_SUCCESS) return false;
  hsa_status_t st = REAL_HSA(hsa_amd_svm_prefetch_async)((void*)p, n, agent, 0, nullptr, sig);
  bool ok = st == HSA_STATUS_SUCCESS;
  if (ok) {
    hsa_signal_value_t v = REAL_HSA(hsa_signal_wait_scacquire)(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX,
                                                               HSA_WAIT_STATE_BLOCKED);
    ok = v == 0;
  }
  REAL_HSA(hsa_signal_destroy)(sig);
  if (!ok) VLOG_WARN("vmem: prefetch of %llu bytes at %p to %s failed (status %d)", (unsigned long long)n, (void*)p,
                     to_gpu ? "HBM" : "host", (int)st);
  return ok;
}

// Bytes of spilled ranges the pager has moved into HBM on `dev`.
uint64_t promoted_bytes(int dev) {
  uint64_t n = 0;
  std::shared_lock<std::shared_mutex> g(g_tab_mu);
  for (VRange* r : g_tab)
    if (r->dev == dev) n += r->gpu_bytes;
  return n;
}

// amdgpu's own VRAM counters (/sys/bus/pci/devices/<bdf>/mem_info_vram_*):
// they count every VRAM buffer, SVM migrations included.  0 when unreadable.
uint64_t sysfs_vram_free(int dev) {
  static std::mutex mu;
  static std::string dirs[VGPU_MAX_DEVICES];
  static bool tried[VGPU_MAX_DEVICES] = {};
  if (dev < 0 || dev >= VGPU_MAX_DEVICES) return 0;
  std::string dir;
  {
    std::lock_guard<std::mutex> l(mu);
    if (!tried[dev]) {
      tried[dev] = true;
      char bus[64] = {0};
      if (REAL_HIP(hipDeviceGetPCIBusId)(bus, sizeof bus, dev) == hipSuccess) {
        for (char* c = bus; *c; ++c) *c = (char)tolower(*c);
        dirs[dev] = std::string("/sys/bus/pci/devices/") + bus;
      }
    }
    dir = dirs[dev];
  }
  if (dir.empty()) return 0;
  auto rd = [](const std::string& p) -> uint64_t {
    FILE* f = fopen(p.c_str(), "r");
    if (!f) return 0;
    unsigned long long v = 0;
    if (fscanf(f, "%llu", &v) != 1) v = 0;
    fclose(f);
    return v;
  };
  uint64_t total = rd(dir + "/mem_info_vram_total"), used = rd(dir + "/mem_info_vram_used");
  return total > used ? total - used : (total ? 1 : 0);
}

// Physical free HBM of `dev` as the pager must see it.  hipMemGetInfo does
// not count VRAM that KFD SVM migrations took (measured: free unchanged after
// a 4 GiB prefetch into HBM), and a migration into a full device stalls the
// process while KFD evicts its own buffers, so the promoted bytes are taken
// off it and amdgpu's VRAM counters have the last word when readable.
uint64_t hbm_free(int dev) {
  size_t f = 0, t = 0;
  const int cur = tl_device;
  if (cur != dev) (void)REAL_HIP(hipSetDevice)(dev);
  hipError_t rc = REAL_HIP(hipMemGetInfo)(&f, &t);
  if (cur != dev && cur >= 0) (void)REAL_HIP(hipSetDevice)(cur);
  if (rc != hipSuccess) return 0;
  const uint64_t mine = promoted_bytes(dev);
  uint64_t free_b = f > mine ? f - mine : 0;
  if (uint64_t sys = sysfs_vram_free(dev)) free_b = std::min(free_b, sys);
  return free_b;
}

// The pod's physical HBM budget on `dev` (0 = the whole device) and what its
// processes hold in HBM now (every process of the container shares the budget).
uint64_t phys_budget(int dev) {
  State& s = st();
  if (!s.region || dev < 0 || dev >= VGPU_MAX_DEVICES) return 0;
  return __atomic_load_n(&s.region->dev[dev].mem_physical, __ATOMIC_RELAXED);
}

uint64_t pod_resident(int dev) {
  State& s = st();
  return s.region ? region_device_used(s.region, dev) : 0;
}

// ---- plain HBM ahead of managed ranges ----------------------------
// Plain buffers (below the managed size: activations, workspaces, the graph
// pool) are read by nearly every kernel; a managed range's last bytes are read
// once per sweep.  So under a budget the pager reserves the pod's recent
// high-water mark of plain bytes before it places managed bytes: a plain
// allocation that the caching allocator frees and makes again finds its room
// still free instead of taking it back from a range's tail (one move out, one
// back in, per cycle).  The mark is the maximum over the current and the last
// VGPU_VMEM_PLAIN_WINDOW_MS (30 s) window, so a transient peak (model loading)
// stops reserving HBM after at most two windows.
std::atomic<uint64_t> g_plain_peak[VGPU_MAX_DEVICES];
std::atomic<uint64_t> g_plain_prev[VGPU_MAX_DEVICES];

uint64_t plain_now(int dev) {
  const uint64_t all = pod_resident(dev), mine = promoted_bytes(dev);
  return all > mine ? all - mine : 0;
}

void note_plain(int dev) {
  if (dev < 0 || dev >= VGPU_MAX_DEVICES || !phys_budget(dev)) return;
  const uint64_t p = plain_now(dev);
  uint64_t cur = g_plain_peak[dev].load(std::memory_order_relaxed);
  while (p > cur && !g_plain_peak[dev].compare_exchange_weak(cur, p, std::memory_order_relaxed)) {
  }
}

void rotate_plain_window() {
  for (int d = 0; d < VGPU_MAX_DEVICES; ++d) {
    g_plain_prev[d].store(g_plain_peak[d].exchange(0, std::memory_order_relaxed), std::memory_order_relaxed);
    note_plain(d);
  }
}

// HBM of `dev`'s budget that placing managed bytes must leave to plain buffers
// beyond what they hold now.
uint64_t plain_reserve(int dev) {
  if (dev < 0 || dev >= VGPU_MAX_DEVICES) return 0;
  const uint64_t mark = std::max(g_plain_peak[dev].load(std::memory_order_relaxed),
                                 g_plain_prev[dev].load(std::memory_order_relaxed));
  const uint64_t p = plain_now(dev);
  return mark > p ? mark - p : 0;
}

// Bytes that may still become HBM-resident on `dev`: the budget (less the plain
// reserve when managed bytes are placed) and physical HBM beyond the headroom.
uint64_t room_left(int dev, bool managed) {
  uint64_t room = UINT64_MAX;
  if (const uint64_t b = phys_budget(dev)) {
    const uint64_t used = pod_resident(dev) + (managed ? plain_reserve(dev) : 0);
    room = b > used ? b - used : 0;
    if (!room) return 0;
  }
  const uint64_t f = hbm_free(dev), h = knobs().headroom;
  return std::min(room, f > h ? f - h : 0);
}

// `need` more bytes may become HBM-resident on `dev`.
bool room_for(int dev, uint64_t need, bool managed = true) { return room_left(dev, managed) >= need; }

// Move the whole range back to host memory.  Caller holds g_move_mu.
bool demote_locked(VRange* r) {
  if (!r->gpu_bytes) return true;
  uint64_t n = r->gpu_bytes;
  auto t0 = std::chrono::steady_clock::now();
  if (!prefetch(r->base, n, r->dev, false)) return false;
  uint64_t ns = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
  r->gpu_bytes = 0;
  r->pager_owned_gpu = false;
  book_move(r->dev, n, false);
  g_out_bytes.fetch_add(n);
  g_moves.fetch_add(1);
  trace_emit(VGPU_EV_MIGRATE, r->dev, n, ns << 1);
  VLOG_INFO("vmem: demoted %llu bytes at %p in %.3f s", (unsigned long long)n, (void*)r->base, ns / 1e9);
  return true;
}

// Promote the next piece of `r`.  Caller holds g_move_mu.  False when there is no room.
// A piece that does not fit whole is cut to the room left, in whole 2 MiB
// granules (KFD's migration granule), so the budget fills up: the resident set
// can then match a zero-copy pod's, which keeps the first budget-full of bytes
// allocated.  The plain reserve keeps later plain buffers from taking that
// room back (the round-3 attempt without it cycled tails out and in).
bool promote_piece_locked(VRange* r) {
  const Knobs& k = knobs();
  constexpr uint64_t kGranule = 2ull << 20;
  uint64_t n = std::min<uint64_t>(k.piece, r->size - r->gpu_bytes);
  if (!n) return false;
  if (!room_for(r->dev, n)) {  // make_room_locked ran first
    if (!k.cut_pieces) return false;
    n = room_left(r->dev, true) & ~(kGranule - 1);
    if (!n) return false;
  }
  auto t0 = std::chrono::steady_clock::now();
  if (!prefetch(r->base + r->gpu_bytes, n, r->dev, true)) return false;
  uint64_t ns = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
  r->gpu_bytes += n;
  r->pager_owned_gpu = true;
  book_move(r->dev, n, true);
  g_in_bytes.fetch_add(n);
  g_moves.fetch_add(1);
  trace_emit(VGPU_EV_MIGRATE, r->dev, n, (ns << 1) | 1);
  VLOG_INFO("vmem: promoted %llu bytes at %p in %.3f s", (unsigned long long)n, (void*)(r->base + r->gpu_bytes - n),
            ns / 1e9);
  return true;
}

// Demote cold promoted ranges of `dev` (oldest first, never `keep`) until
// `need` bytes of HBM are free beyond the headroom.  Caller holds g_move_mu.
bool make_room_locked(int dev, uint64_t need, const VRange* keep, uint64_t newer_than, bool managed = true) {
  if (room_for(dev, need, managed)) return true;
  std::vector<VRange*> cold;
  {
    std::shared_lock<std::shared_mutex> g(g_tab_mu);
    for (VRange* r : g_tab)
      if (r != keep && r->dev == dev && r->gpu_bytes && r->last_use.load() < newer_than) cold.push_back(r);
  }
  std::sort(cold.begin(), cold.end(), [](VRange* a, VRange* b) { return a->last_use.load() < b->last_use.load(); });
  for (VRange* r : cold) {
    if (room_for(dev, need, managed)) break;
    demote_locked(r);
  }
  return room_for(dev, need, managed);
}

// Suspended (SIGUSR2): give back every byte of HBM our managed ranges hold.
// Runs on the pager thread; in-flight work is safe (KFD pauses the queues).
void evict_all() {
  std::lock_guard<std::mutex> m(g_move_mu);
  std::vector<VRange*> held;
  {
    std::shared_lock<std::shared_mutex> g(g_tab_mu);
    for (VRange* r : g_tab)
      if (r->gpu_bytes) held.push_back(r);
  }
  uint64_t n = 0;
  for (VRange* r : held) {  // g_move_mu keeps vmem_release out: the pointers stay valid
    n += r->gpu_bytes;
    demote_locked(r);
  }
  if (n) VLOG_INFO("vmem: suspended, %llu bytes of HBM released to host memory", (unsigned long long)n);
}

void pager_step(bool advance) {
  const Knobs& k = knobs();
  const uint64_t tick = advance ? g_tick.fetch_add(1) + 1 : g_tick.load();
  if (advance && tick % (1000 / k.tick_ms + 1) == 0) {
    std::shared_lock<std::shared_mutex> g(g_tab_mu);
    for (VRange* r : g_tab) r->uses.store(r->uses.load() / 2);
  }
  if (advance) {
    if (tick % std::max<uint64_t>(1, k.plain_window_ms / k.tick_ms) == 0) rotate_plain_window();
    bool seen[VGPU_MAX_DEVICES] = {};
    {
      std::shared_lock<std::shared_mutex> g(g_tab_mu);
      for (VRange* r : g_tab)
        if (r->dev >= 0 && r->dev < VGPU_MAX_DEVICES) seen[r->dev] = true;
    }
    for (int d = 0; d < VGPU_MAX_DEVICES; ++d)
      if (seen[d]) note_plain(d);
  }
  // Snapshot the candidates by value under the table lock: a concurrent
  // hipFree (vmem_release) may delete a range as soon as the lock is dropped,
  // so a pointer is dereferenced again only after re-checking membership
  // under g_move_mu (which vmem_release also holds).
  struct Cand {
    VRange* r;
    uint32_t uses;
  };
  std::vector<Cand> hot;
  {
    std::shared_lock<std::shared_mutex> g(g_tab_mu);
    for (VRange* r : g_tab)
      if (r->gpu_bytes < r->size && r->last_use.load() + k.hot_ticks >= tick && r->last_use.load())
        hot.push_back({r, r->uses.load()});
  }
  if (hot.empty()) return;
  std::sort(hot.begin(), hot.end(), [](const Cand& a, const Cand& b) { return a.uses > b.uses; });
  uint64_t waiting = 0;
  int waiting_dev = -1;
  for (const Cand& c : hot) {
    VRange* r = c.r;
    std::lock_guard<std::mutex> m(g_move_mu);
    {  // freed meanwhile?
      std::shared_lock<std::shared_mutex> g(g_tab_mu);
      if (std::find(g_tab.begin(), g_tab.end(), r) == g_tab.end()) continue;
    }
    // Room for a hot range may come from any range that is not hot itself
    // (unused for the hot window): hot ranges are never exchanged for each
    // other, but a model whose traffic stopped a second ago gives way at once
    // instead of after the 2 s cold window that new allocations wait for
    // (a model switch started promoting one second earlier).
    // While a launch is gated on this promotion, its graph's ranges carry the
    // gate's tick and everything older is idle: it may give way at once.
    const uint64_t stale = std::max(tick > k.hot_ticks ? tick - k.hot_ticks : 0, g_gate_tick.load());
    while (r->gpu_bytes < r->size) {
      uint64_t n = std::min<uint64_t>(k.piece, r->size - r->gpu_bytes);
      (void)make_room_locked(r->dev, n, r, stale);  // what it could not free, a cut piece may still use
      if (!promote_piece_locked(r)) {
        waiting += r->size - r->gpu_bytes;
        waiting_dev = r->dev;
        break;
      }
    }
  }
  static uint64_t last_note = 0;
  if (waiting && advance && tick - last_note >= 1000 / (uint64_t)k.tick_ms) {
    last_note = tick;
    VLOG_INFO("vmem: %llu bytes of used spilled ranges wait for HBM (free for the pager %llu)",
              (unsigned long long)waiting, (unsigned long long)hbm_free(waiting_dev));
  }
}

void drain_repairs();

void pager_main() {
  pthread_setname_np(pthread_self(), "vgpu-vmem");
  tl_device = -1;
  // HIP calls from this thread must not invalidate another thread's stream capture.
  hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
  (void)REAL_HIP(hipThreadExchangeStreamCaptureMode)(&mode);
  const Knobs& k = knobs();
  std::unique_lock<std::mutex> l(g_thr_mu);
  bool evicted = false;
  auto last = std::chrono::steady_clock::now();
  while (g_thr_run) {
    // Poll every millisecond for a launch that named a non-resident range
    // (promotion starts then, not at the next tick); the tick itself, which
    // ages use counts and measures hot/cold windows, advances every tick_ms.
    g_thr_cv.wait_for(l, std::chrono::milliseconds(1));
    if (!g_thr_run) break;
    l.unlock();
    drain_repairs();
    l.lock();
    const auto now = std::chrono::steady_clock::now();
    const bool tick = now - last >= std::chrono::milliseconds(k.tick_ms);
    const bool woke = g_wake.exchange(0) != 0;
    if (!tick && !woke) continue;
    if (tick) last = now;
    l.unlock();
    if (st().suspended.load(std::memory_order_relaxed)) {
      if (!evicted && g_count.load() > 0) evict_all();
      evicted = true;
    } else {
      evicted = false;
      if (g_count.load() > 0) pager_step(tick);
    }
    l.lock();
  }
  g_thr_alive.store(0);
}

void ensure_pager() {
  std::lock_guard<std::mutex> l(g_thr_mu);
  if (g_thr_run) return;
  g_thr_run = true;
  g_thr_alive.store(1);
  std::thread(pager_main).detach();
}

}  // namespace

// Oversubscribed pods spill before the device is physically full: the HIP
// runtime and ROCr still need HBM of their own after the application's last
// buffer (code objects loaded lazily at a kernel's first launch, scratch,
// kernarg pools) and fail with hipErrorNoBinaryForGpu / out-of-resources
// when it is gone.  VGPU_VMEM_RESERVE_MB (default 1024) stays free.
bool vmem_should_spill(int dev, uint64_t size) {
  static const uint64_t reserve = [] {
    const char* e = env_first("VGPU_VMEM_RESERVE_MB");
    return (e ? strtoull(e, nullptr, 10) : 1024ull) << 20;
  }();
  // Called after `size` was reserved against the cap, so the pod's resident
  // bytes already include it.
  // The budget yields to an open graph capture: its (small, graph-pool)
  // buffers can neither become managed ranges nor pinned host memory while a
  // global-mode capture is open, so they stay plain HBM; the cap still holds.
  const uint64_t b = phys_budget(dev);
  if (b && pod_resident(dev) > b && g_open_captures.load(std::memory_order_acquire) == 0) return true;
  return hbm_free(dev) < size + reserve;
}

bool vmem_wants_managed(int dev, uint64_t size) {
  const Knobs& k = knobs();
  // Not while a graph capture is open: hipMemAdvise would be an unsafe call in
  // a global-mode capture.  Those (activation) buffers take the plain path.
  return vmem_enabled() && k.managed_min >= 0 && (uint64_t)k.managed_min <= size &&
         (phys_budget(dev) > 0 || k.suspend_evict) && g_open_captures.load(std::memory_order_acquire) == 0;
}

bool vmem_enabled() {
  State& s = st();
  return s.enabled && s.region && (s.region->oversubscribe || knobs().suspend_evict) && knobs().on;
}

namespace {
VRange* new_range(void** ptr, size_t size, int dev, hipError_t* rc) {
  *rc = REAL_HIP(hipMallocManaged)(ptr, size, hipMemAttachGlobal);
  if (*rc != hipSuccess) return nullptr;
  // Coarse-grained: coherent at kernel boundaries like hipMalloc memory, so
  // the GPU caches it (fine-grained managed memory bypasses them).
  (void)REAL_HIP(hipMemAdvise)(*ptr, size, hipMemAdviseSetCoarseGrain, dev);
  (void)REAL_HIP(hipGetLastError)();
  // Host-resident parts are read in place over the host link; 2 MiB host pages
  // let the GPU map them with larger fragments (fewer translation misses).
  if (knobs().thp) (void)madvise(*ptr, size, MADV_HUGEPAGE);
  auto* r = new VRange((uintptr_t)*ptr, size, dev);
  r->last_use.store(g_tick.load());  // allocated now: in use now
  {
    std::unique_lock<std::shared_mutex> g(g_tab_mu);
    g_tab.insert(std::upper_bound(g_tab.begin(), g_tab.end(), r,
                                  [](const VRange* a, const VRange* b) { return a->base < b->base; }),
                 r);
    g_count.store((int)g_tab.size());
  }
  ensure_pager();
  return r;
}
}  // namespace

hipError_t vmem_alloc_overflow(void** ptr, size_t size, int dev) {
  if (!vmem_enabled()) return hipErrorNotSupported;
  hipError_t rc;
  return new_range(ptr, size, dev, &rc) ? hipSuccess : rc;
}

hipError_t vmem_alloc_managed(void** ptr, size_t size, int dev) {
  if (!vmem_enabled()) return hipErrorNotSupported;
  hipError_t rc;
  VRange* r = new_range(ptr, size, dev, &rc);
  if (!r) return rc;
  // Resident at once while the budget has room (after cold ranges made way);
  // the rest, if any, is promoted by the pager once the range is in use.
  const Knobs& k = knobs();
  std::lock_guard<std::mutex> m(g_move_mu);
  const uint64_t tick = g_tick.load();
  const uint64_t stale = tick > k.cold_ticks ? tick - k.cold_ticks : 0;
  while (r->gpu_bytes < r->size) {
    const uint64_t n = std::min<uint64_t>(k.piece, r->size - r->gpu_bytes);
    (void)make_room_locked(dev, n, r, stale);
    if (!promote_piece_locked(r)) break;
  }
  return hipSuccess;
}

// ---- host copies ---------------------------------------------------------------------
// hipMemcpy* between host memory and a managed range is carried out on the
// host side: KFD migrates every page the copy touches to system memory first,
// whatever the copy kind, pinned or pageable, sync or async (measured:
// native/probes/managed_access.hip -- a promoted 512 MiB range reads at
// 57 GB/s after one hipMemcpy into it, 6.1 TB/s before).  Those pages never
// come back by themselves (XNACK off: the GPU reads them over the host link)
// and the pager's books still call the range resident, so it would never
// promote them either -- a VGG-16 pod whose weights were uploaded with
// model.to("cuda") ran its FC GEMMs 55x slower.  After such a copy, the
// resident part of each range it touched goes back to HBM, whole 2 MiB
// granules at a time (KFD's migration granule).  hooks_hip.cpp avoids most of
// this by staging such copies through plain HBM (device-to-device copies leave
// the pages where they are); this is the fallback (open captures, no staging).
namespace {
struct Span {
  uintptr_t lo = 0;
  uint64_t n = 0;
  int dev = -1;
};

Span resident_span_locked(const void* p, size_t n) {
  VRange* r = find_locked((uintptr_t)p);
  if (!r || !r->gpu_bytes || !n) return {};
  constexpr uintptr_t g = 2ull << 20;
  const uintptr_t lo = std::max<uintptr_t>(r->base, (uintptr_t)p & ~(g - 1));
  const uintptr_t hi = std::min<uintptr_t>(r->base + r->gpu_bytes, ((uintptr_t)p + n + g - 1) & ~(g - 1));
  return hi > lo ? Span{lo, hi - lo, r->dev} : Span{};
}
}  // namespace

int vmem_resident_dev(const void* p, size_t n) {
  if (g_count.load(std::memory_order_relaxed) == 0) return -1;
  std::shared_lock<std::shared_mutex> g(g_tab_mu);
  const Span s = resident_span_locked(p, n);
  return s.n ? s.dev : -1;
}

bool vmem_copy_touches(const void* dst, const void* src, size_t n) {
  if (g_count.load(std::memory_order_relaxed) == 0) return false;
  std::shared_lock<std::shared_mutex> g(g_tab_mu);
  return resident_span_locked(dst, n).n || resident_span_locked(src, n).n;
}

void vmem_after_copy(const void* dst, const void* src, size_t n) {
  if (g_count.load(std::memory_order_relaxed) == 0) return;
  std::lock_guard<std::mutex> m(g_move_mu);  // no demotion in between
  Span sp[2];
  {
    std::shared_lock<std::shared_mutex> g(g_tab_mu);
    sp[0] = resident_span_locked(dst, n);
    sp[1] = resident_span_locked(src, n);
  }
  for (const Span& s : sp) {
    if (!s.n) continue;
    auto t0 = std::chrono::steady_clock::now();
    if (!prefetch(s.lo, s.n, s.dev, true)) continue;
    uint64_t ns = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    trace_emit(VGPU_EV_MIGRATE, s.dev, s.n, (ns << 1) | 1);
    VLOG_DEBUG("vmem: %llu bytes at %p back to HBM after a host copy (%.3f s)", (unsigned long long)s.n,
               (void*)s.lo, ns / 1e9);
  }
}

// Async copies and memsets that touched a resident range without staging: the
// repair (vmem_after_copy) waits for the operation on the pager thread behind an
// event recorded on its stream, so the caller's stream stays asynchronous
// (it used to hipStreamSynchronize in the caller).
namespace {
// The resident spans the operation touched, as of queueing.  At drain time
// they are cut to what is still resident under g_move_mu:
// meanwhile the pager or vmem_make_room may have demoted the range, a
// suspend-evict moved it to host, or hipFree released it -- prefetching the
// queued spans whole would pull stale pages back into HBM behind the books.
// A span never grows at drain time: the pager's later promotions are its own
// (a grown span re-migrated pages a kernel was writing, round 5 vmemcopy).
struct Repair {
  hipEvent_t ev;
  Span sp[2];
};
std::mutex g_rep_mu;
std::vector<Repair> g_rep;
std::atomic<int> g_rep_n{0};

void drain_repairs() {
  if (g_rep_n.load(std::memory_order_relaxed) == 0) return;
  std::vector<Repair> done;
  {
    std::lock_guard<std::mutex> l(g_rep_mu);
    for (auto it = g_rep.begin(); it != g_rep.end();) {
      const hipError_t q = REAL_HIP(hipEventQuery)(it->ev);
      if (q == hipErrorNotReady) {
        ++it;
        continue;
      }
      done.push_back(*it);
      it = g_rep.erase(it);
    }
    g_rep_n.store((int)g_rep.size(), std::memory_order_relaxed);
  }
  (void)REAL_HIP(hipGetLastError)();
  for (Repair& r : done) {
    (void)REAL_HIP(hipEventDestroy)(r.ev);
    std::lock_guard<std::mutex> m(g_move_mu);
    if (st().suspended.load(std::memory_order_relaxed)) continue;  // suspend-evict owns the placement now
    Span sp[2];
    {
      std::shared_lock<std::shared_mutex> g(g_tab_mu);
      for (int k = 0; k < 2; ++k) {
        const Span& q = r.sp[k];
        if (!q.n) continue;
        const Span now = resident_span_locked((const void*)q.lo, q.n);  // released ranges: no span
        const uintptr_t lo = std::max(q.lo, now.lo), hi = std::min(q.lo + q.n, now.lo + now.n);
        if (now.n && hi > lo && now.dev == q.dev) sp[k] = Span{lo, hi - lo, q.dev};
      }
    }
    for (const Span& s : sp)
      if (s.n && prefetch(s.lo, s.n, s.dev, true)) {
        trace_emit(VGPU_EV_MIGRATE, s.dev, s.n, 1);
        VLOG_DEBUG("vmem: %llu bytes at %p back to HBM after an async copy", (unsigned long long)s.n, (void*)s.lo);
      }
  }
}
}  // namespace

bool vmem_after_copy_async(const void* dst, const void* src, size_t n, hipStream_t stream) {
  if (g_count.load(std::memory_order_relaxed) == 0) return true;
  Repair r{};
  {
    std::shared_lock<std::shared_mutex> g(g_tab_mu);
    r.sp[0] = resident_span_locked(dst, n);
    r.sp[1] = resident_span_locked(src, n);
  }
  if (!r.sp[0].n && !r.sp[1].n) return true;
  if (REAL_HIP(hipEventCreateWithFlags)(&r.ev, hipEventDisableTiming) != hipSuccess) {
    (void)REAL_HIP(hipGetLastError)();
    return false;
  }
  if (REAL_HIP(hipEventRecord)(r.ev, stream) != hipSuccess) {
    (void)REAL_HIP(hipGetLastError)();
    (void)REAL_HIP(hipEventDestroy)(r.ev);
    return false;
  }
  ensure_pager();
  std::lock_guard<std::mutex> l(g_rep_mu);
  g_rep.push_back(r);
  g_rep_n.store((int)g_rep.size(), std::memory_order_relaxed);
  return true;
}

bool vmem_owns(void* p) {
  if (g_count.load(std::memory_order_relaxed) == 0) return false;
  std::shared_lock<std::shared_mutex> g(g_tab_mu);
  VRange* r = find_locked((uintptr_t)p);
  return r && r->base == (uintptr_t)p;
}

bool vmem_contains(const void* p) {
  if (g_count.load(std::memory_order_relaxed) == 0) return false;
  std::shared_lock<std::shared_mutex> g(g_tab_mu);
  return find_locked((uintptr_t)p) != nullptr;
}

bool vmem_release(void* p) {
  if (!vmem_owns(p)) return false;
  std::lock_guard<std::mutex> m(g_move_mu);
  VRange* r = nullptr;
  {
    std::unique_lock<std::shared_mutex> g(g_tab_mu);
    auto it = std::find_if(g_tab.begin(), g_tab.end(), [&](VRange* x) { return x->base == (uintptr_t)p; });
    if (it == g_tab.end()) return false;
    r = *it;
    g_tab.erase(it);
    g_count.store((int)g_tab.size());
  }
  // the ledger books the whole allocation as host bytes: book the HBM part back first
  if (r->gpu_bytes) {
    vgpu_proc_slot_t* sl = my_slot();
    if (sl && r->dev >= 0 && r->dev < VGPU_MAX_DEVICES) {
      vgpu_dev_usage_t& u = sl->used[r->dev];
      __atomic_fetch_sub(&u.buffer_bytes, r->gpu_bytes, __ATOMIC_RELAXED);
      __atomic_fetch_sub(&u.total_bytes, r->gpu_bytes, __ATOMIC_RELAXED);
      __atomic_fetch_add(&u.host_bytes, r->gpu_bytes, __ATOMIC_RELAXED);
    }
  }
  delete r;
  return true;
}

// Move the last `n` resident bytes of `r` back to host memory (the resident
// part stays a prefix).  Caller holds g_move_mu.
static bool demote_tail_locked(VRange* r, uint64_t n) {
  n = std::min(n, r->gpu_bytes);
  if (!n) return false;
  auto t0 = std::chrono::steady_clock::now();
  if (!prefetch(r->base + r->gpu_bytes - n, n, r->dev, false)) return false;
  uint64_t ns = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
  r->gpu_bytes -= n;
  book_move(r->dev, n, false);
  g_out_bytes.fetch_add(n);
  g_moves.fetch_add(1);
  trace_emit(VGPU_EV_MIGRATE, r->dev, n, ns << 1);
  VLOG_INFO("vmem: %llu tail bytes of the range at %p to host memory for a plain allocation",
            (unsigned long long)n, (void*)r->base);
  return true;
}

bool vmem_make_room(int dev, uint64_t need) {
  if (g_count.load(std::memory_order_relaxed) == 0) return false;
  std::lock_guard<std::mutex> m(g_move_mu);
  const Knobs& k = knobs();
  const uint64_t tick = g_tick.load();
  if (make_room_locked(dev, need, nullptr, tick > k.cold_ticks ? tick - k.cold_ticks : 0, false)) return true;
  // Nothing is cold and the budget is full of managed ranges.  An allocation
  // below the managed size is activation / workspace sized and used by every
  // kernel that follows: spilled, each of them would cross the host link.  It
  // takes its room from the tail of the largest resident range instead, which
  // kernels then read in place (a part E pod spilled 11 such buffers, ~190 MB,
  // behind 11.8 GB of resident weights).  The caller has reserved `need`.
  const uint64_t b = phys_budget(dev);
  if (!b || k.managed_min < 0 || need >= (uint64_t)k.managed_min) return false;
  constexpr uint64_t g = 2ull << 20;
  while (pod_resident(dev) > b) {
    VRange* big = nullptr;
    {
      std::shared_lock<std::shared_mutex> gl(g_tab_mu);
      for (VRange* r : g_tab)
        if (r->dev == dev && r->gpu_bytes && (!big || r->gpu_bytes > big->gpu_bytes)) big = r;
    }
    if (!big || !demote_tail_locked(big, (pod_resident(dev) - b + g - 1) & ~(g - 1))) return false;
  }
  return true;
}

// The application's own hipMemPrefetchAsync.  A prefetch is a hint, so the
// shim may shorten it.  Into a range the pager owns it does nothing: the pager
// keeps the books of what is resident, and pages moved behind its back would
// never be promoted again (to host) or would overrun the budget (to HBM).
// Elsewhere a prefetch into HBM is cut to the HBM free beyond the headroom, in
// whole 2 MiB granules.  Asked to migrate more than is free, KFD makes room by
// evicting the process's own buffers (profiles/vmem_r2.md: pages that stay on
// the host, one run hung); hbm_free() counts SVM pages (sysfs VRAM counters),
// which hipMemGetInfo does not, so the cut holds with a small headroom.
size_t vmem_prefetch_allowed(const void* p, size_t n, int dev) {
  if (vmem_contains(p)) return 0;
  if (dev < 0) return n;
  const uint64_t f = hbm_free(dev), h = knobs().headroom;
  const uint64_t room = f > h ? (f - h) & ~((2ull << 20) - 1) : 0;
  return (size_t)std::min<uint64_t>(n, room);
}

void vmem_note_plain(int dev) {
  if (g_count.load(std::memory_order_relaxed) == 0) return;
  note_plain(dev);
}

namespace {
// Graph bookkeeping: ranges named by launches captured into a graph, keyed by
// capture id while the capture is open, then by graph, then by executable.
std::mutex g_gmu;
std::unordered_map<unsigned long long, std::vector<uintptr_t>> g_cap_ranges;
std::unordered_map<const void*, std::vector<uintptr_t>> g_graph_ranges;
std::unordered_map<const void*, std::vector<uintptr_t>> g_exec_ranges;

void merge(std::vector<uintptr_t>& into, const std::vector<uintptr_t>& from) {
  into.insert(into.end(), from.begin(), from.end());
  std::sort(into.begin(), into.end());
  into.erase(std::unique(into.begin(), into.end()), into.end());
}

// Capture id of `stream` when it is being captured, else 0.
unsigned long long capture_id(hipStream_t stream) {
  if (g_open_captures.load(std::memory_order_acquire) == 0) return 0;
  auto info = REAL_HIP(hipStreamGetCaptureInfo);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  if (!info || info(stream, &cs, &id) != hipSuccess || cs != hipStreamCaptureStatusActive) return 0;
  return id ? id : 1;
}

// Runs `scan` (which stamps ranges); when `stream` is capturing, the ranges
// it names are also recorded for the graph being captured.
template <class F>
void scan_for(hipStream_t stream, F&& scan) {
  const unsigned long long cid = capture_id(stream);
  if (!cid) {
    scan();
  } else {
    std::vector<uintptr_t> hits;
    tl_sink = &hits;
    scan();
    tl_sink = nullptr;
    if (!hits.empty()) {
      std::lock_guard<std::mutex> l(g_gmu);
      merge(g_cap_ranges[cid], hits);
    }
  }
  if (g_wake.load(std::memory_order_relaxed)) g_thr_cv.notify_one();
}
}  // namespace

namespace {
// The argument values of a launch (an array of pointers to them, as
// hipLaunchKernel takes it): [lo, hi) is the part of the calling thread's
// stack above the scanner; arrays or values outside it are not read (their
// sizes are unknown, so nothing bounds a read there).  Sorted addresses bound
// each value by the next one.
template <class F>
void with_arg_values(void** args, uintptr_t lo, uintptr_t hi, F&& each) {
  if ((uintptr_t)args < lo || (uintptr_t)args >= hi) return;  // not a stub frame: nothing safe to read
  uintptr_t a[64];
  int n = 0;
  for (int i = 0; i < 64; ++i) {
    if ((uintptr_t)(args + i) + sizeof(void*) > hi) break;
    uintptr_t e = (uintptr_t)args[i];
    if (e < lo || e + sizeof(uint32_t) > hi) break;
    a[n++] = e;
  }
  if (!n) return;
  std::sort(a, a + n);
  for (int i = 0; i < n; ++i) {
    // The last argument's size is unknown: a bounded look (PyTorch's
    // elementwise kernels pass their operand pointer array last).
    uintptr_t end = i + 1 < n ? a[i + 1] : a[i] + 512;
    end = std::min<uintptr_t>({end, a[i] + 4096, hi});
    if (end > a[i]) each(a[i], end - a[i]);
  }
}

// The kernarg buffer of a module launch's `extra` (HIP_LAUNCH_PARAM_BUFFER_*), bounded.
bool extra_buffer(void** extra, const void** buf, size_t* n) {
  *buf = nullptr;
  *n = 0;
  for (int i = 0; extra && i < 8 && extra[i] != HIP_LAUNCH_PARAM_END; i += 2) {
    if (extra[i] == HIP_LAUNCH_PARAM_BUFFER_POINTER) *buf = extra[i + 1];
    else if (extra[i] == HIP_LAUNCH_PARAM_BUFFER_SIZE && extra[i + 1]) *n = *(size_t*)extra[i + 1];
  }
  *n = std::min<size_t>(*n, 4096);
  return *buf && *n;
}
}  // namespace

void vmem_scan_args(void** args, hipStream_t stream) {
  if (g_count.load(std::memory_order_relaxed) == 0 || !args) return;
  const uintptr_t lo = (uintptr_t)__builtin_frame_address(0);
  const uintptr_t hi = stack_top();
  scan_for(stream, [&] {
    const uint64_t tick = g_tick.load(std::memory_order_relaxed);
    std::shared_lock<std::shared_mutex> g(g_tab_mu);
    if (g_tab.empty()) return;
    with_arg_values(args, lo, hi, [&](uintptr_t p, size_t n) { scan_words_locked((const unsigned char*)p, n, tick); });
  });
}

void vmem_scan_extra(void** extra, hipStream_t stream) {
  if (g_count.load(std::memory_order_relaxed) == 0 || !extra) return;
  const void* buf;
  size_t n;
  if (!extra_buffer(extra, &buf, &n)) return;
  scan_for(stream, [&] {
    const uint64_t tick = g_tick.load(std::memory_order_relaxed);
    std::shared_lock<std::shared_mutex> g(g_tab_mu);
    if (!g_tab.empty()) scan_words_locked((const unsigned char*)buf, n, tick);
  });
}

// A copy engine operation (peer copy) that reads or writes [p, p+n): the
// ranges it touches are in use, as if a kernel had named them.
void vmem_note_use(const void* p, hipStream_t stream) {
  if (g_count.load(std::memory_order_relaxed) == 0 || !p) return;
  scan_for(stream, [&] {
    const uint64_t tick = g_tick.load(std::memory_order_relaxed);
    std::shared_lock<std::shared_mutex> g(g_tab_mu);
    if (!g_tab.empty()) touch_word((uintptr_t)p, tick);
  });
}

unsigned long long vmem_capture_begin_id(hipStream_t stream) { return capture_id(stream); }

void vmem_capture_ended(unsigned long long cid, hipGraph_t graph) {
  if (!cid) return;
  std::lock_guard<std::mutex> l(g_gmu);
  auto it = g_cap_ranges.find(cid);
  if (it == g_cap_ranges.end()) return;
  if (graph) merge(g_graph_ranges[graph], it->second);
  g_cap_ranges.erase(it);
}

void vmem_graph_instantiated(hipGraph_t graph, hipGraphExec_t exec) {
  std::lock_guard<std::mutex> l(g_gmu);
  auto it = g_graph_ranges.find(graph);
  if (it == g_graph_ranges.end()) {
    g_exec_ranges.erase(exec);
    return;
  }
  g_exec_ranges[exec] = it->second;
}

void vmem_graph_destroyed(const void* graph_or_exec) {
  {
    std::lock_guard<std::mutex> l(g_gmu);
    g_graph_ranges.erase(graph_or_exec);
    g_exec_ranges.erase(graph_or_exec);
  }
  std::lock_guard<std::mutex> l(g_nogate_mu);
  g_nogate.erase(graph_or_exec);
}

// Explicitly built graphs (hipGraphAdd*Node, *SetParams, hipGraphExec*SetParams):
// the ranges a node's kernel arguments or copy / memset pointers name join
// the graph's (or executable's) set, as captured launches do.
void vmem_graph_note(const void* key, bool exec, void** args, void** extra, const void* const* ptrs, int nptrs) {
  if (g_count.load(std::memory_order_relaxed) == 0 || !key) return;
  const uintptr_t lo = (uintptr_t)__builtin_frame_address(0);
  const uintptr_t hi = stack_top();
  std::vector<uintptr_t> hits;
  {
    std::shared_lock<std::shared_mutex> g(g_tab_mu);
    if (g_tab.empty()) return;
    tl_sink = &hits;
    tl_collect_only = true;
    if (args) with_arg_values(args, lo, hi, [&](uintptr_t p, size_t n) { scan_words_locked((const unsigned char*)p, n, 0); });
    const void* buf;
    size_t n;
    if (extra && extra_buffer(extra, &buf, &n)) scan_words_locked((const unsigned char*)buf, n, 0);
    for (int i = 0; i < nptrs; ++i)
      if (ptrs[i]) touch_word((uintptr_t)ptrs[i], 0);
    tl_collect_only = false;
    tl_sink = nullptr;
  }
  if (hits.empty()) return;
  std::sort(hits.begin(), hits.end());
  hits.erase(std::unique(hits.begin(), hits.end()), hits.end());
  std::lock_guard<std::mutex> l(g_gmu);
  merge(exec ? g_exec_ranges[key] : g_graph_ranges[key], hits);
}

void vmem_graph_child(hipGraph_t graph, hipGraph_t child) {
  std::lock_guard<std::mutex> l(g_gmu);
  auto it = g_graph_ranges.find(child);
  if (it != g_graph_ranges.end() && !it->second.empty()) {
    const std::vector<uintptr_t> c = it->second;  // merge may rehash the map
    merge(g_graph_ranges[graph], c);
  }
}

// A replay runs none of our hooks: stamp every range its kernels name.
namespace {
// Bytes of the graph's ranges (all, and not in HBM) and their device.
void graph_bytes(const std::vector<uintptr_t>& bases, uint64_t* total, uint64_t* host, int* dev) {
  *total = *host = 0;
  *dev = -1;
  std::shared_lock<std::shared_mutex> g(g_tab_mu);
  if (g_tab.empty()) return;
  for (uintptr_t b : bases)
    if (VRange* r = find_locked(b)) {
      *total += r->size;
      *host += r->size - std::min<uint64_t>(r->gpu_bytes, r->size);
      *dev = r->dev;
    }
}
}  // namespace

// A replayed graph runs no hooks, so its ranges are stamped here.  If most of
// them are on the host (a model switch back: part D), the launch waits for the
// pager first: replays reading over the host link while KFD pauses the queues
// for every migration piece ran both slowly — promotion at 1.5 GB/s beside the
// replays against 7 GB/s alone, a 10 s switch (profiles/r4/vmem/part_d_*).
// Only graphs whose ranges fit the budget beside the plain buffers are gated
// (a hot set beyond the budget — part E — is read in place, never waited
// for), at most VGPU_VMEM_GATE_MS (0: never), and an executable whose gate
// made no progress for a second is not gated again.
void vmem_graph_launched(hipGraphExec_t exec) {
  if (g_count.load(std::memory_order_relaxed) == 0) return;
  std::vector<uintptr_t> bases;
  {
    std::lock_guard<std::mutex> l(g_gmu);
    auto it = g_exec_ranges.find(exec);
    if (it == g_exec_ranges.end()) return;
    bases = it->second;
  }
  const Knobs& k = knobs();
  constexpr uint64_t kGateMin = 1ull << 30;  // gate a launch with this much of its graph on the host
  constexpr uint64_t kGateEnd = 64ull << 20;  // and let it go once less is left (the last piece, cut)
  uint64_t total = 0, host = 0;
  int dev = -1;
  bool gate = false;
  if (k.gate_ms && k.on && !st().suspended.load(std::memory_order_relaxed)) {
    graph_bytes(bases, &total, &host, &dev);
    if (host >= kGateMin && dev >= 0) {
      const uint64_t b = phys_budget(dev), plain = plain_now(dev);
      const uint64_t room = b ? (b > plain ? b - plain : 0) : UINT64_MAX;
      std::lock_guard<std::mutex> l(g_nogate_mu);
      gate = total <= room && !g_nogate.count(exec);
    }
  }
  // A gated launch stamps its ranges one tick ahead, so whatever ran before
  // it is older than the gate.
  const uint64_t tick = gate ? g_tick.fetch_add(1) + 1 : g_tick.load(std::memory_order_relaxed);
  {
    std::shared_lock<std::shared_mutex> g(g_tab_mu);
    if (g_tab.empty()) return;
    for (uintptr_t b : bases) touch_word(b, tick);
  }
  if (g_wake.load(std::memory_order_relaxed)) g_thr_cv.notify_one();
  if (!gate) return;
  uint64_t expected = 0;
  g_gate_tick.compare_exchange_strong(expected, tick);
  const auto t0 = std::chrono::steady_clock::now();
  auto t_prog = t0;
  uint64_t left = host;
  bool done = false;
  VLOG_INFO("vmem: launch waits for %llu bytes of its graph's ranges to reach HBM", (unsigned long long)host);
  auto t_stamp = t0;
  while (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(k.gate_ms)) {
    g_wake.store(1, std::memory_order_relaxed);
    g_thr_cv.notify_one();
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
    if (std::chrono::steady_clock::now() - t_stamp > std::chrono::milliseconds(100)) {
      // still in use: keep the graph's ranges inside the pager's hot window
      t_stamp = std::chrono::steady_clock::now();
      const uint64_t now_tick = g_tick.load(std::memory_order_relaxed);
      std::shared_lock<std::shared_mutex> g(g_tab_mu);
      if (!g_tab.empty())
        for (uintptr_t b : bases) touch_word(b, now_tick);
    }
    uint64_t tot2, h2;
    int d2;
    graph_bytes(bases, &tot2, &h2, &d2);
    if (h2 < kGateEnd) {
      done = true;
      break;
    }
    const auto now = std::chrono::steady_clock::now();
    if (h2 < left) {
      left = h2;
      t_prog = now;
    } else if (now - t_prog > std::chrono::milliseconds(1000 + (int64_t)k.hot_ticks * k.tick_ms)) {
      break;  // no room to be had: read in place from now on
    }
  }
  expected = tick;
  g_gate_tick.compare_exchange_strong(expected, 0);
  if (!done) {
    std::lock_guard<std::mutex> l(g_nogate_mu);
    g_nogate.insert(exec);
  }
  VLOG_INFO("vmem: gated launch went on after %.3f s (%llu bytes still on the host)",
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(), (unsigned long long)left);
}

uint64_t vmem_graph_ranges(hipGraphExec_t exec) {
  std::lock_guard<std::mutex> l(g_gmu);
  auto it = g_exec_ranges.find(exec);
  return it == g_exec_ranges.end() ? 0 : it->second.size();
}

void vmem_book_move(int dev, uint64_t bytes, bool to_gpu) { book_move(dev, bytes, to_gpu); }

void vmem_stats(uint64_t* in_bytes, uint64_t* out_bytes, uint64_t* moves, uint64_t* gpu_bytes,
                uint64_t* ranges) {
  *in_bytes = g_in_bytes.load();
  *out_bytes = g_out_bytes.load();
  *moves = g_moves.load();
  uint64_t gb = 0;
  std::shared_lock<std::shared_mutex> g(g_tab_mu);
  for (VRange* r : g_tab) gb += r->gpu_bytes;
  *gpu_bytes = gb;
  *ranges = g_tab.size();
}

// The budget's books on `dev`: budget, pod resident, this process's managed
// bytes in HBM, plain bytes, plain reserve, managed bytes on the host,
// managed ranges larger than 1 GiB partly in HBM, physical free HBM.
void vmem_budget_books(int dev, uint64_t out[8]) {
  for (int i = 0; i < 8; ++i) out[i] = 0;
  if (dev < 0 || dev >= VGPU_MAX_DEVICES) return;
  out[0] = phys_budget(dev);
  out[1] = pod_resident(dev);
  out[2] = promoted_bytes(dev);
  out[3] = plain_now(dev);
  out[4] = plain_reserve(dev);
  std::shared_lock<std::shared_mutex> g(g_tab_mu);
  for (VRange* r : g_tab) {
    if (r->dev != dev) continue;
    out[5] += r->size - r->gpu_bytes;
    out[6] += r->gpu_bytes && r->gpu_bytes < r->size;
  }
  g.unlock();
  out[7] = hbm_free(dev);
}

void vmem_stop() {
  {
    std::lock_guard<std::mutex> l(g_thr_mu);
    if (!g_thr_run) return;
    g_thr_run = false;
  }
  g_thr_cv.notify_all();
  // let a migration in flight finish before the runtime is torn down
  for (int i = 0; i < 500 && g_thr_alive.load(); ++i) std::this_thread::sleep_for(std::chrono::milliseconds(10));
}

void vmem_after_fork() {
  // The pager thread does not exist in the child.  Mutexes may have been held
  // by it at fork time: re-create them.
  new (&g_thr_mu) std::mutex();
  new (&g_move_mu) std::mutex();
  new (&g_tab_mu) std::shared_mutex();
  new (&g_gmu) std::mutex();
  g_thr_run = false;
  g_thr_alive.store(0);
}

}  // namespace vgpu
