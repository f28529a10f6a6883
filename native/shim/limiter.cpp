// Compute-share enforcement on the dispatch path.
//
// Reference behaviour: libvgpu.so's
// `utilization_watcher` thread samples per-process SM utilization
// (nvmlDeviceGetProcessUtilization) every 120 ms and feeds a global token
// counter; `rate_limiter(grids, blocks)` runs on every cuLaunchKernel: it
// blocks while the monitor has set recent_kernel < 0 (priority preemption),
// sets recent_kernel = 2, returns when the limit is 0 or >= 100 or
// utilizationSwitch == 0, and otherwise CAS-decrements the counter by `grids`,
// sleeping while it is negative.
//
// MI355X design.  The PRIMARY mechanism is spatial (XCD-balanced CU masks on
// every HSA queue, cumask.cpp): exact and free per dispatch.  This temporal
// limiter engages when a mask cannot express the share
// (GPU_CORE_UTILIZATION_POLICY=force, VGPU_CU_MASK_FROM_LIMIT=false, or more
// sharers than a GPU has good mask slots for).  ROCm has no per-process
// busy-time counter for KFD user queues (KFD's cu_occupancy is an occupancy
// snapshot, not time), so the limiter measures the GPU time of its OWN work:
//
//   * after every tracked launch (kernel, module kernel, graph) the hook
//     records a timing-free marker event on the launch's stream and pushes it
//     onto the launching thread's own ring (one single-producer /
//     single-consumer ring per thread and device: no lock and no shared
//     read-modify-write on the launch path — the reference's rate_limiter is
//     one CAS per cuLaunchKernel, SURVEY.md §3.5 hot loop #1);
//   * the limiter thread drains the rings (hipEventQuery, 100 µs) and turns
//     "this process had work outstanding on the device from t0 to t1" into a
//     charge.  With a share board (board.cpp; node-wide, one per GPU) the
//     charge is the processor-sharing virtual time of the interval — each of k
//     concurrently busy pods pays 1/k of the wall time — otherwise it is the
//     wall time itself;
//   * a token bucket in GPU-nanoseconds refills at limit% of wall time, and
//     the launch hook blocks while the bucket, minus the estimated cost of the
//     work already in flight, is negative.
//
// The charge is for time actually spent on the GPU, so it is exact for a
// graph replay as for a stream of tiny kernels, needs no host-PID mapping,
// and converges on hardware without calibration.
#include <dlfcn.h>
#include <fcntl.h>
#include <math.h>
#include <strings.h>
#include <sys/stat.h>

#include <condition_variable>
#include <thread>
#include <unordered_map>
#include <vector>

#include "board.h"
#include "common.h"
#include "real.h"
#include "state.h"

namespace vgpu {

thread_local int tl_device = 0;
thread_local int tl_in_hip_alloc = 0;
std::atomic<int> g_open_captures{0};
std::shared_mutex g_capture_mu;

extern int cumask_device_cus(int dev);        // CUs available to us (mask or physical)
extern uint32_t cumask_driver_uid(int dev);   // KFD gpu_id of device, 0 = unknown
extern int cumask_device_physical_cus(int dev);

namespace {

// ---- per-thread marker rings -----------------------------------------------------------
constexpr uint32_t kRing = 1024;  // markers in flight per thread and device (power of two)
constexpr uint32_t kMask = kRing - 1;

struct Marker {
  hipEvent_t ev;
  uint64_t submit_ns;
  hipStream_t stream;
  uint32_t launches;  // launches this marker covers
};

// One launching thread's markers on one device.  The thread (producer) writes
// ring[head], the limiter thread (consumer) retires ring[tail] once its event
// has completed and hands the event back through `fring` for reuse.
struct Track {
  // producer side
  alignas(64) std::atomic<uint32_t> head{0};
  std::atomic<uint32_t> ftail{0};     // next free event to take (producer advances)
  std::atomic<uint64_t> launches{0};  // tracked launches, monotonic (owner stores only)
  hipEvent_t spare = nullptr;         // an event whose record failed, reused next time
  // consumer side
  alignas(64) std::atomic<uint32_t> tail{0};
  std::atomic<uint32_t> fhead{0};     // free events handed back (consumer advances)
  std::atomic<uint64_t> pub_seen{0};  // `launches` when the consumer last published inflight
  uint64_t charged = 0;               // launches retired (consumer only)
  std::atomic<int> dead{0};           // the owning thread exited
  Marker ring[kRing];
  hipEvent_t fring[kRing];
};

std::atomic<uint32_t> g_track_gen{1};  // bumped at fork: the child's thread-local tracks are stale

struct DevLimiter {
  int active = 0;             // temporal limiting configured for this device
  double frac = 0;            // share of the time this process may have work on the device
  std::atomic<int> pool_scale_pending{0};  // frac still to be scaled by device CUs / pool CUs
  std::atomic<int64_t> tokens{0};  // fair-share GPU ns we may still spend
  int64_t cap = 0;            // bucket depth (ns)
  int64_t quantum = 0;        // an overdrawn bucket must refill this far before launches resume
  std::atomic<int> hold{0};   // 1 while waiting for the quantum
  std::atomic<int64_t> inflight_pub{0};  // tracked launches not yet charged, as of the last drain
  std::atomic<int64_t> ema_charge{0};    // charged ns per launch
  std::atomic<int> idle{1};   // consumer: nothing outstanding (a producer that sees it wakes the thread)
  std::atomic<int> busy{0};   // consumer: a busy interval is open (act_mark_ns valid)
  std::mutex tracks_mu;       // guards `tracks` (registration; the consumer's pass)
  std::vector<Track*> tracks;
  std::mutex mu;              // guards act_mark_ns / board attach
  uint64_t act_mark_ns = 0;   // start of the not-yet-charged busy interval
  uint64_t activated_ns = 0;  // last (re-)activation: markers from before are not charged
  uint64_t interval_charge = 0;  // charged since the previous marker completion (per-launch estimate)
  uint64_t last_poll_ns = 0;  // previous poll that found work still in flight
  vgpu_board_t* board = nullptr;
  int board_slot = -1;
  bool board_tried = false;
  std::atomic<int> board_ready{0};  // attach_board ran (the launch path checks this without the lock)
  // Concurrency gate of the temporal pool (VGPU_POOL_CONCURRENCY, 0 = off): at
  // most max_running pool members of the GPU run at once, in run_quantum_ns turns.
  int max_running = 0;
  uint64_t run_quantum_ns = 0;
  // window statistics (limiter thread only)
  uint64_t win_charge = 0, win_busy = 0, win_start = 0;
  std::atomic<uint64_t> charged_total{0}, busy_total{0};
  // Adaptive share policy (VGPU_CU_SHARE=auto): dispatch sizes of the last
  // window, and whether this process holds CUs of its own (spatial mode).
  int auto_share = 0;
  std::atomic<uint64_t> kern_n{0};  // dispatches since the last auto_step (graph launch = 1), batched per thread
  int spatial = 0;
  bool auto_joined = false;
  bool pool0_saved = false;
  uint64_t pool0[VGPU_CU_MASK_WORDS] = {};  // the plugin's pool mask (all-zero = every CU)
  uint32_t pool_gen = 0;                    // the plugin's mask-write generation pool0 was taken at
  // Marker-independent busy check: KFD's cu_occupancy of this
  // process on the device, sampled every occ_period_ns.  A sample with waves on
  // the CUs counts the time since the previous sample as busy; every window the
  // busy time the samples saw beyond what the markers charged is charged too, so
  // work whose markers complete early (a profiler rewriting completion signals:
  // 3.4 x the share under rocprofv3, profiles/r3/temporal) still pays.
  int occ_fd = -2;                 // -2 not opened yet, -1 unavailable
  uint64_t occ_next_try_ns = 0;
  uint64_t occ_last_ns = 0, occ_window_start = 0;
  uint64_t occ_busy_acc = 0;       // busy wall the samples saw in this window
  uint64_t occ_mark_acc = 0;       // wall the markers charged in this window (reaped intervals)
  uint64_t occ_credit = 0;         // in-flight interval time already credited to the previous window
  std::atomic<uint64_t> untracked_ns{0};  // last launch the markers deliberately do not charge
  std::atomic<uint64_t> occ_extra_total{0};  // charged on the occupancy evidence alone
  // What this process last saw or wrote in the region's mask (its own CAS
  // writes and sibling processes' writes); pool0 changes only when the device
  // plugin's generation in the region's flags moves (custate.py _reshape_pool).
  uint64_t shim_mask[VGPU_CU_MASK_WORDS] = {};
};

DevLimiter g_lim[VGPU_MAX_DEVICES];
std::atomic<int> g_throttle_any{0};
std::atomic<int> g_auto_any{0};
std::atomic<int> g_thread_running{0};
std::atomic<int> g_shutdown{0};
std::atomic<int> g_thread_alive{0};
std::mutex g_cv_mu;
std::condition_variable g_cv;

// Debt is bounded: tokens never fall below -(cap + 1 s), so a
// replay of up to a second is still paid in full while no accumulation of
// charges can hold a pod for longer than that debt's refill.
void charge_tokens(DevLimiter& L, int64_t ns) {
  if (ns <= 0) return;
  const int64_t floor = -(L.cap + 1000000000ll);
  int64_t cur = L.tokens.load(std::memory_order_relaxed), nv;
  do {
    nv = cur - ns;
    if (nv < floor) nv = floor;
  } while (!L.tokens.compare_exchange_weak(cur, nv, std::memory_order_relaxed));
}

// The calling thread's track for `dev` (created and registered on first use).
struct ThreadTracks {
  Track* t[VGPU_MAX_DEVICES] = {};
  uint32_t gen = 0;
  ~ThreadTracks() {
    if (gen != g_track_gen.load(std::memory_order_relaxed)) return;  // stale copy (forked child)
    for (Track* x : t)
      if (x) x->dead.store(1, std::memory_order_release);  // the limiter thread frees it once drained
  }
};
thread_local ThreadTracks tl_tracks;

Track* my_track(int dev) {
  ThreadTracks& tt = tl_tracks;
  const uint32_t gen = g_track_gen.load(std::memory_order_relaxed);
  if (__builtin_expect(tt.gen != gen, 0)) {
    for (auto& x : tt.t) x = nullptr;  // forked: the parent's rings are not ours (leaked in the child)
    tt.gen = gen;
  }
  Track* t = tt.t[dev];
  if (__builtin_expect(t != nullptr, 1)) return t;
  t = new Track();
  DevLimiter& L = g_lim[dev];
  {
    std::lock_guard<std::mutex> g(L.tracks_mu);
    L.tracks.push_back(t);
  }
  tt.t[dev] = t;
  return t;
}

// Launches this thread made on `dev` that the last drain had not seen yet.
int64_t own_unpublished(int dev) {
  Track* t = tl_tracks.t[dev];
  if (!t || tl_tracks.gen != g_track_gen.load(std::memory_order_relaxed)) return 0;
  return (int64_t)(t->launches.load(std::memory_order_relaxed) - t->pub_seen.load(std::memory_order_relaxed));
}

// Per-thread batching of the region slot's counters and the auto policy's
// dispatch count: a launch touches no cache line another thread writes.
struct ThreadCounts {
  uint64_t launches = 0, kern[VGPU_MAX_DEVICES] = {};
  uint64_t last_flush_ns = 0;
  uint32_t since = 0;
};
thread_local ThreadCounts tl_counts;

void flush_counts(ThreadCounts& c, uint64_t now) {
  if (vgpu_proc_slot_t* sl = my_slot()) {
    if (c.launches) __atomic_fetch_add(&sl->launches, c.launches, __ATOMIC_RELAXED);
    __atomic_store_n(&sl->last_launch_ns, now, __ATOMIC_RELAXED);
  }
  c.launches = 0;
  for (int d = 0; d < VGPU_MAX_DEVICES; ++d)
    if (c.kern[d]) {
      g_lim[d].kern_n.fetch_add(c.kern[d], std::memory_order_relaxed);
      c.kern[d] = 0;
    }
  c.since = 0;
  c.last_flush_ns = now;
}

const char* lock_dir() {
  const char* d = env_first("VGPU_LOCK_DIR");
  return d && *d ? d : "/tmp/vgpulock";
}

// Board of the physical GPU behind logical device `dev` (lazy; caller holds L.mu).
void attach_board(int dev, DevLimiter& L) {
  if (L.board_tried) return;
  L.board_tried = true;
  if (!env_bool(env_first("VGPU_SHARE_BOARD"), true)) return;
  State& s = st();
  char key[VGPU_UUID_LEN + 16] = {};
  if (s.region && s.region->dev[dev].uuid[0])
    snprintf(key, sizeof key, "%s", s.region->dev[dev].uuid);
  else if (uint32_t uid = cumask_driver_uid(dev))
    snprintf(key, sizeof key, "kfd-%u", uid);
  else
    return;
  for (char* p = key; *p; ++p)
    if (*p == '/') *p = '_';
  struct stat stt;
  if (stat(lock_dir(), &stt) != 0 || !S_ISDIR(stt.st_mode)) return;
  char path[640];
  // Layout version in the name: shims of different board layouts never share
  // a mapping during a rolling upgrade.
  snprintf(path, sizeof path, "%s/%s.v%u.board", lock_dir(), key, (unsigned)VGPU_BOARD_VERSION);
  L.board = board_map(path);
  if (!L.board) return;
  L.board_slot = board_claim(L.board, getpid(), self_host_pid(nullptr), (int)lround(L.frac * 100));
  if (L.board_slot < 0) {
    VLOG_WARN("share board %s is full; charging wall time", path);
    L.board = nullptr;
    return;
  }
  VLOG_INFO("device %d: fair-share board %s slot %d", dev, path, L.board_slot);
}

// A pool member's limit is a share of the whole device, but its work only
// runs on the pool's CUs: a 25 % vGPU on a 128-CU pool of a 256-CU device may
// keep the pool busy 50 % of the time.  Needs the HSA agents (first launch).
void apply_pool_scale(int dev, DevLimiter& L) {
  int expected = 1;
  if (!L.pool_scale_pending.compare_exchange_strong(expected, 0)) return;
  State& s = st();
  int pool = 0;
  for (int w = 0; w < VGPU_CU_MASK_WORDS; ++w)
    pool += __builtin_popcountll(__atomic_load_n(&s.region->dev[dev].cu_mask[w], __ATOMIC_RELAXED));
  const int phys = cumask_device_physical_cus(dev);
  if (pool <= 0 || phys <= 0 || pool >= phys) return;
  const double f = fmin(1.0, L.frac * phys / pool);
  VLOG_INFO("device %d: pool of %d/%d CUs, time share %.0f%% -> %.0f%%", dev, pool, phys, 100 * L.frac, 100 * f);
  const double r = f / L.frac;
  L.frac = f;
  L.cap = (int64_t)(L.cap * r);
  L.quantum = (int64_t)(L.quantum * r);
  L.tokens.store(L.cap);
}

uint32_t pool_gen_of(const vgpu_device_cfg_t& d) {
  return (__atomic_load_n(&d.flags, __ATOMIC_ACQUIRE) >> VGPU_DEV_POOL_GEN_SHIFT) & 0xffffu;
}

// Decide per device whether temporal throttling applies.
void configure() {
  State& s = st();
  int any = 0;
  for (int d = 0; d < VGPU_MAX_DEVICES; ++d) {
    uint32_t lim = s.region ? s.region->dev[d].cu_limit : s.lim.cu_limit[d];
    bool has_mask = false;
    if (s.region)
      for (int w = 0; w < VGPU_CU_MASK_WORDS; ++w) has_mask |= s.region->dev[d].cu_mask[w] != 0;
    const char* share = env_first("VGPU_CU_SHARE");
    // VGPU_CU_SHARE=temporal (device plugin, pool member): the share is
    // enforced in time; a mask, if any, is the pool of CUs the pool members share.
    // VGPU_CU_SHARE=auto: the same, until the process's dispatches turn out
    // too small to fill the GPU; then it claims CUs of its own (auto_step).
    const bool auto_share = share && !strcasecmp(share, "auto");
    const bool temporal_share = auto_share || (share && !strcasecmp(share, "temporal"));
    bool want = lim > 0 && lim < 100 && s.lim.core_policy != 2;
    DevLimiter& La = g_lim[d];
    if (auto_share && want) {
      La.auto_share = 1;
      if (!La.pool0_saved && s.region) {
        for (int w = 0; w < VGPU_CU_MASK_WORDS; ++w)
          La.shim_mask[w] = La.pool0[w] = __atomic_load_n(&s.region->dev[d].cu_mask[w], __ATOMIC_RELAXED);
        La.pool_gen = pool_gen_of(s.region->dev[d]);
        La.pool0_saved = true;
      }
      g_auto_any.store(1, std::memory_order_relaxed);
    }
    if (La.auto_share && La.spatial) want = false;  // own CUs: the mask is the share
    if (!temporal_share) {
      // A CU mask already enforces the share spatially; temporal limiting on
      // top of it only when explicitly forced.
      if (has_mask && s.lim.core_policy != 1) want = false;
      if (!has_mask && s.lim.core_policy == 0 && env_bool(env_first("VGPU_CU_MASK_FROM_LIMIT"), true))
        want = false;  // cumask.cpp derives a balanced mask from the limit
    }
    DevLimiter& L = g_lim[d];
    if (want && !L.active) {
      L.frac = lim / 100.0;
      L.pool_scale_pending.store(temporal_share && has_mask && !L.auto_share ? 1 : 0);
      const double burst_ms = env_first("VGPU_LIMITER_BURST_MS") ? atof(env_first("VGPU_LIMITER_BURST_MS")) : 50.0;
      L.cap = (int64_t)(L.frac * burst_ms * 1e6);
      // Time-slice quantum: a throttled pod runs in slices of ~quantum_ms of
      // wall time (at its share) instead of one launch per refill, so the
      // per-slice costs (clock ramp after idle, pipeline fill) are amortised.
      const double q_ms = env_first("VGPU_LIMITER_QUANTUM_MS") ? atof(env_first("VGPU_LIMITER_QUANTUM_MS")) : 200.0;
      L.quantum = (int64_t)(L.frac * q_ms * 1e6);
      // Concurrency gate: several pods whose kernels each fill the GPU slow each
      // other down more than time-slicing does (caches, HBM pages, CP queue
      // switching), so a pool member may be held until fewer than N run.
      const char* mr = env_first("VGPU_POOL_CONCURRENCY");
      L.max_running = temporal_share && mr ? atoi(mr) : 0;
      const char* rq = env_first("VGPU_POOL_QUANTUM_MS");
      L.run_quantum_ns = (uint64_t)((rq ? atof(rq) : 50.0) * 1e6);
      if (L.cap < L.quantum) L.cap = L.quantum;
      L.tokens.store(L.cap);
      L.win_start = mono_ns();
      // Re-activated (an auto member back from CUs of its own): markers left
      // from before were not reaped meanwhile, so the busy interval and the
      // board's fair-share mark still date from then.  Charging that whole gap
      // on the first poll overdrew the bucket and held the pod through the
      // next time-shared window (its A/B/A windows disagreed 2:1, profiles/r4).
      std::lock_guard<std::mutex> g(L.mu);
      const uint64_t now = mono_ns();
      L.act_mark_ns = L.last_poll_ns = L.activated_ns = now;
      L.occ_last_ns = L.occ_window_start = now;
      L.occ_busy_acc = L.occ_mark_acc = L.occ_credit = 0;
      if (L.board) (void)board_charge(L.board, L.board_slot, 0, !L.busy.load());
    }
    L.active = want;
    any |= want;
  }
  g_throttle_any.store(any, std::memory_order_release);
}

// True while `stream` is being captured into a graph (a marker recorded or
// queried there would join or invalidate the capture).
bool stream_capturing(hipStream_t stream) {
  if (g_open_captures.load(std::memory_order_acquire) == 0) return false;
  auto is_cap = REAL_HIP(hipStreamIsCapturing);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return !is_cap || is_cap(stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone;
}

// Hand a completed marker's event back to its producer (or destroy it when
// the producer's free ring is full).
void recycle_event(Track* t, hipEvent_t ev) {
  const uint32_t fh = t->fhead.load(std::memory_order_relaxed);
  if (fh - t->ftail.load(std::memory_order_acquire) >= kRing) {
    (void)REAL_HIP(hipEventDestroy)(ev);
    return;
  }
  t->fring[fh & kMask] = ev;
  t->fhead.store(fh + 1, std::memory_order_release);
}

void free_track(Track* t) {
  const uint32_t fh = t->fhead.load(std::memory_order_acquire);
  for (uint32_t i = t->ftail.load(std::memory_order_acquire); i != fh; ++i) (void)REAL_HIP(hipEventDestroy)(t->fring[i & kMask]);
  if (t->spare) (void)REAL_HIP(hipEventDestroy)(t->spare);
  delete t;
}

// Drain the rings of `dev`: retire completed markers, charge the busy wall
// time since the previous charge, publish the in-flight launch count.
//
// The whole pass runs under the capture guard (shared): hipStreamBeginCapture
// (exclusive) waits for a pass in progress, and no pass starts while a capture
// is being opened.  Without it a pass that passed the open-captures check could
// query a marker of a stream whose capture began a moment later, and the
// runtime invalidates that capture (seen on MI355X: a torch graph capture on a
// stream with markers from its eager warm-up failed at its first kernel with
// hipErrorStreamCaptureInvalidated).
bool reap(int dev, DevLimiter& L) {
  std::shared_lock<std::shared_mutex> cap(g_capture_mu);
  auto query = REAL_HIP(hipEventQuery);
  int done = 0, left = 0;
  int64_t covered = 0, inflight = 0;
  uint64_t first_submit = UINT64_MAX;  // oldest marker not retired before this pass
  std::vector<Track*> gone;
  {
    std::lock_guard<std::mutex> g(L.tracks_mu);
    for (size_t i = 0; i < L.tracks.size();) {
      Track* t = L.tracks[i];
      uint32_t tl = t->tail.load(std::memory_order_relaxed);
      const uint32_t h = t->head.load(std::memory_order_acquire);
      if (tl != h && t->ring[tl & kMask].submit_ns < first_submit) first_submit = t->ring[tl & kMask].submit_ns;
      uint64_t cov = 0;
      while (tl != h) {
        Marker& m = t->ring[tl & kMask];
        // A stream being captured is polled after its capture ends.
        if (stream_capturing(m.stream)) break;
        const hipError_t rc = query(m.ev);
        if (rc == hipErrorNotReady || rc == hipErrorStreamCaptureUnsupported || rc == hipErrorStreamCaptureImplicit)
          break;
        recycle_event(t, m.ev);  // complete (or invalid: never wait on it again)
        cov += m.launches;
        ++tl;
        ++done;
      }
      t->tail.store(tl, std::memory_order_release);
      t->charged += cov;
      covered += (int64_t)cov;
      left += (int)(h - tl);
      const uint64_t produced = t->launches.load(std::memory_order_relaxed);
      inflight += (int64_t)(produced - t->charged);
      t->pub_seen.store(produced, std::memory_order_relaxed);
      if (tl == h && t->dead.load(std::memory_order_acquire) && t->head.load(std::memory_order_acquire) == tl) {
        gone.push_back(t);
        L.tracks[i] = L.tracks.back();
        L.tracks.pop_back();
        continue;
      }
      ++i;
    }
  }
  for (Track* t : gone) free_track(t);
  L.inflight_pub.store(inflight > 0 ? inflight : 0, std::memory_order_relaxed);
  const uint64_t polled = mono_ns();
  std::lock_guard<std::mutex> g(L.mu);
  if (!done && !left) return false;
  if (!L.busy.load(std::memory_order_relaxed)) {
    // Idle -> busy: the interval starts at the oldest marker's submission.
    attach_board(dev, L);
    L.act_mark_ns = first_submit < polled ? first_submit : polled;
    if (L.act_mark_ns < L.activated_ns) L.act_mark_ns = L.activated_ns;
    L.last_poll_ns = polled;
    L.busy.store(1, std::memory_order_relaxed);
    if (L.board) board_enter(L.board, L.board_slot);
  }
  uint64_t now;
  if (!done) {
    // Still running: charge the busy time so far every 2 ms instead of in one
    // lump at completion, so the bucket drains while a long replay runs and
    // its refill is not lost to the bucket's cap (a 350 ms replay against a
    // 100 ms bucket ran at 0.4 of a 0.5 share), and the occupancy cross-check
    // compares like with like.
    L.last_poll_ns = polled;
    if (polled - L.act_mark_ns < 2000000ull) return true;
    now = polled;
  } else {
    // The completion happened between the previous poll and this one.
    now = L.last_poll_ns > L.act_mark_ns ? (L.last_poll_ns + polled) / 2 : polled;
    if (now < L.act_mark_ns) now = L.act_mark_ns;
    L.last_poll_ns = polled;
  }
  const uint64_t wall = now > L.act_mark_ns ? now - L.act_mark_ns : 0;
  L.act_mark_ns = now;
  const uint64_t charge = L.board ? board_charge(L.board, L.board_slot, wall, done && left == 0) : wall;
  charge_tokens(L, (int64_t)charge);
  L.interval_charge += charge;
  if (done) {
    // per-launch cost estimate from everything charged since the previous completion
    const int64_t per = covered > 0 ? (int64_t)(L.interval_charge / covered) : (int64_t)L.interval_charge;
    const int64_t old = L.ema_charge.load(std::memory_order_relaxed);
    L.ema_charge.store(old ? (old * 3 + per) / 4 : per, std::memory_order_relaxed);
    L.interval_charge = 0;
  }
  L.win_charge += charge;
  L.win_busy += wall;
  L.occ_mark_acc += wall;
  L.charged_total.fetch_add(charge, std::memory_order_relaxed);
  L.busy_total.fetch_add(wall, std::memory_order_relaxed);
  trace_emit(VGPU_EV_GPU_TIME, dev, charge, wall);
  if (left == 0) {
    L.busy.store(0, std::memory_order_relaxed);
    // Publish idleness, then look once more: a producer that pushed before
    // the store may not have seen it (and did not wake us).
    L.idle.store(1, std::memory_order_seq_cst);
  }
  return left > 0;
}

// Any marker waiting in a ring of `dev`.
bool rings_pending(DevLimiter& L) {
  std::lock_guard<std::mutex> g(L.tracks_mu);
  for (Track* t : L.tracks)
    if (t->tail.load(std::memory_order_relaxed) != t->head.load(std::memory_order_acquire)) return true;
  return false;
}

// The auto policy's write of its own mask: word by word, only over the value
// it last saw (compare-and-swap), so a pool reshape the device plugin wrote
// meanwhile wins and is picked up at the next step.  Returns false when the
// region changed under us.
bool write_own_mask(int dev, DevLimiter& L, const uint64_t m[VGPU_CU_MASK_WORDS]) {
  State& s = st();
  if (!s.region) return false;
  bool ok = true;
  for (int w = 0; w < VGPU_CU_MASK_WORDS; ++w) {
    uint64_t expect = L.shim_mask[w];
    if (__atomic_compare_exchange_n(&s.region->dev[dev].cu_mask[w], &expect, m[w], false, __ATOMIC_RELAXED,
                                    __ATOMIC_RELAXED))
      L.shim_mask[w] = m[w];
    else
      ok = false;  // external value stays; shim_mask keeps the old one so the next step sees the change
  }
  return ok;
}

// Adaptive share policy (VGPU_CU_SHARE=auto; the device plugin's default).
// Measured on MI355X (docs/benchmarks.md): four 25 % pods of ResNet-50
// inference (dispatches of thousands of workgroups) run 1.7 x faster time-shared
// than on CU masks of their own -- a masked queue's CUs idle while the CP
// time-slices it against another queue -- while ResNet-152 training, DeepLab
// training and the LSTMs run 1.2-1.35 x faster on masks, and no per-dispatch
// statistic the shim can see separates the two groups (scripts/kernel_sizes.py,
// profiles/r3/policy).  So the pods of a GPU measure both: the share board runs
// an A/B (board_auto_lead) -- a window time-shared, a window with every busy
// member on an XCD-balanced claim of its share's CUs -- compares each member's
// dispatch rate and keeps whichever was faster on average (re-measured when
// the set of busy members changes, or every VGPU_AUTO_REEXPLORE_S).  A member
// on its own CUs runs unthrottled; the other members of the GPU's pool shrink
// to the CUs nobody claimed.
void auto_step() {
  State& s = st();
  static const uint64_t window_ns = (uint64_t)(1e6 * (env_first("VGPU_AUTO_WINDOW_MS") ? atof(env_first("VGPU_AUTO_WINDOW_MS")) : 1500.0));
  static const uint64_t settle_ns = (uint64_t)(1e6 * (env_first("VGPU_AUTO_SETTLE_MS") ? atof(env_first("VGPU_AUTO_SETTLE_MS")) : 300.0));
  static const uint64_t reexplore_ns = (uint64_t)(1e9 * (env_first("VGPU_AUTO_REEXPLORE_S") ? atof(env_first("VGPU_AUTO_REEXPLORE_S")) : 300.0));
  static const double min_gain = env_first("VGPU_AUTO_MIN_GAIN") ? atof(env_first("VGPU_AUTO_MIN_GAIN")) : 1.05;
  static const uint64_t bucket_ns = (uint64_t)(1e6 * (env_first("VGPU_AUTO_BUCKET_MS") ? atof(env_first("VGPU_AUTO_BUCKET_MS")) : 1000.0));
  for (int d = 0; d < VGPU_MAX_DEVICES; ++d) {
    DevLimiter& L = g_lim[d];
    if (!L.auto_share || !s.region) continue;
    {
      std::lock_guard<std::mutex> g(L.mu);
      attach_board(d, L);
    }
    if (!L.board) continue;
    if (!L.auto_joined) {
      board_auto_join(L.board, L.board_slot);
      L.auto_joined = true;
    }
    board_auto_progress(L.board, L.board_slot, L.kern_n.exchange(0, std::memory_order_relaxed));
    char note[160];
    const int phase = board_auto_lead(L.board, L.board_slot, window_ns, settle_ns, reexplore_ns, min_gain, bucket_ns,
                                      note, sizeof note);
    if (note[0]) VLOG_INFO("device %d: adaptive share: %s", d, note);
    const int phys = cumask_device_physical_cus(d);
    // The region's mask is shared by every process of the container: a value
    // we did not write is either a sibling process's (its own claim or reset:
    // adopted as what we last saw, so our CAS writes stay valid) or the device
    // plugin's pool reshape, which moves the generation in the region's flags
    // (reading every foreign value as a reshape made siblings adopt
    // each other's claims as their pool).  A reshape is the pool from now on; a
    // claim we held is given up and re-made from the new pool at a later step.
    {
      uint64_t cur[VGPU_CU_MASK_WORDS];
      for (int w = 0; w < VGPU_CU_MASK_WORDS; ++w) cur[w] = __atomic_load_n(&s.region->dev[d].cu_mask[w], __ATOMIC_RELAXED);
      const uint32_t gen = pool_gen_of(s.region->dev[d]);
      if (gen != L.pool_gen) {
        L.pool_gen = gen;
        for (int w = 0; w < VGPU_CU_MASK_WORDS; ++w) L.shim_mask[w] = L.pool0[w] = cur[w];
        int n = 0;
        for (int w = 0; w < VGPU_CU_MASK_WORDS; ++w) n += __builtin_popcountll(cur[w]);
        VLOG_INFO("device %d: adaptive share: pool reshaped by the device plugin to %d CUs", d, n ? n : phys);
        if (L.spatial) {
          uint64_t none[4], full_pool[VGPU_CU_MASK_WORDS];
          for (int w = 0; w < VGPU_CU_MASK_WORDS; ++w) full_pool[w] = ~0ull;
          board_claim_cus(L.board, L.board_slot, 0, 8, full_pool, none);
          L.spatial = 0;
          trace_emit(VGPU_EV_QUEUE, d, 0, 0);
        }
      } else {
        for (int w = 0; w < VGPU_CU_MASK_WORDS; ++w) L.shim_mask[w] = cur[w];
      }
    }
    uint64_t allowed[VGPU_CU_MASK_WORDS];
    bool any = false;
    for (int w = 0; w < VGPU_CU_MASK_WORDS; ++w) any |= L.pool0[w] != 0;
    for (int w = 0; w < VGPU_CU_MASK_WORDS; ++w) {
      const int lo = 64 * w;
      const uint64_t full = phys <= lo ? 0 : (phys >= lo + 64 ? ~0ull : ((1ull << (phys - lo)) - 1));
      allowed[w] = any ? L.pool0[w] : full;
    }
    const bool want_own = (phase == VGPU_AUTO_EXPLORE_S || phase == VGPU_AUTO_SPATIAL) && s.region->proc_num <= 1;
    if (want_own && !L.spatial) {
      const uint32_t nx = 8;
      const uint32_t lim = s.region->dev[d].cu_limit;
      const uint32_t want = ((uint32_t)((phys > 0 ? phys : 256) * lim + 99) / 100 + nx - 1) / nx * nx;
      uint64_t got[4];
      if (board_claim_cus(L.board, L.board_slot, want, nx, allowed, got)) {
        if (write_own_mask(d, L, got)) {
          L.spatial = 1;
          trace_emit(VGPU_EV_QUEUE, d, 1, want);
        } else {
          uint64_t none[4];
          board_claim_cus(L.board, L.board_slot, 0, 8, allowed, none);  // pool changed meanwhile
        }
      }
      continue;
    }
    if (!want_own && L.spatial) {
      uint64_t none[4];
      board_claim_cus(L.board, L.board_slot, 0, 8, allowed, none);
      L.spatial = 0;
      trace_emit(VGPU_EV_QUEUE, d, 0, 0);
    }
    if (L.spatial) continue;
    // pool member: every allowed CU nobody claimed
    uint64_t others[4], mask[VGPU_CU_MASK_WORDS];
    board_claims_of_others(L.board, L.board_slot, others);
    bool full = true;
    for (int w = 0; w < VGPU_CU_MASK_WORDS; ++w) {
      mask[w] = allowed[w] & ~others[w];
      full &= mask[w] == allowed[w];
    }
    if (full && !any)
      for (int w = 0; w < VGPU_CU_MASK_WORDS; ++w) mask[w] = 0;  // all CUs
    bool same = true;
    for (int w = 0; w < VGPU_CU_MASK_WORDS; ++w) same &= L.shim_mask[w] == mask[w];
    if (!same) (void)write_own_mask(d, L, mask);
  }
}

// ---- occupancy cross-check -------------------------------------------------------------
uint64_t occ_period_ns() {
  static const uint64_t p = (uint64_t)(1e3 * (env_first("VGPU_LIMITER_OCC_US") ? atof(env_first("VGPU_LIMITER_OCC_US"))
                                                                                  : 2000.0));
  return p;  // 0 disables the check
}

int occ_open(int dev, DevLimiter& L, uint64_t now) {
  if (L.occ_fd != -2 && L.occ_fd != -1) return L.occ_fd;
  if (L.occ_fd == -1 && now < L.occ_next_try_ns) return -1;
  L.occ_next_try_ns = now + 500000000ull;  // host pid / KFD entry may appear later: look again in 0.5 s
  L.occ_fd = -1;
  int src = 0;
  int pid = self_host_pid(&src);
  if (src == VGPU_HOSTPID_UNVERIFIED) {
    vgpu_proc_slot_t* sl = my_slot();
    if (!sl || __atomic_load_n(&sl->host_pid_src, __ATOMIC_ACQUIRE) == VGPU_HOSTPID_UNVERIFIED) return -1;
    pid = __atomic_load_n(&sl->host_pid, __ATOMIC_RELAXED);
  }
  const uint32_t uid = cumask_driver_uid(dev);
  if (pid <= 0 || !uid) return -1;
  char path[512];
  snprintf(path, sizeof path, "%s/%d/stats_%u/cu_occupancy", kfd_proc_dir(), pid, uid);
  const int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd >= 0) {
    L.occ_fd = fd;
    VLOG_INFO("device %d: limiter cross-checks its markers with %s", dev, path);
  }
  return fd;
}

// Every 100 ms: the busy wall the occupancy samples saw against the wall the
// markers account for in the same window.  The markers' share of a window is
// the reaped intervals plus the interval still in flight up to now, minus the
// in-flight part already credited to the previous window (reap books an
// interval whole when its marker completes, so a replay longer than the window
// is neither charged twice nor missing from the window it ran in).
// Windows in which this process made launches the markers deliberately do not
// charge (launches while the monitor reports no contention) are skipped:
// occupancy cannot tell that work from the rest.
void occ_step(int dev, DevLimiter& L, uint64_t now) {
  const uint64_t period = occ_period_ns();
  if (!period) return;
  if (L.occ_last_ns && now - L.occ_last_ns < period) return;
  const int fd = occ_open(dev, L, now);
  if (fd < 0) return;
  char buf[32];
  const ssize_t n = pread(fd, buf, sizeof buf - 1, 0);
  if (n <= 0) return;
  buf[n] = 0;
  const long occ = strtol(buf, nullptr, 10);
  const uint64_t dt = L.occ_last_ns ? std::min<uint64_t>(now - L.occ_last_ns, 2 * period) : 0;
  L.occ_last_ns = now;
  if (occ > 0) L.occ_busy_acc += dt;
  if (!L.occ_window_start) L.occ_window_start = now;
  static const uint64_t window = 100000000ull;  // reconcile every 100 ms
  if (now - L.occ_window_start < window) return;
  std::lock_guard<std::mutex> g(L.mu);
  const uint64_t inflight = L.busy.load(std::memory_order_relaxed) && now > L.act_mark_ns ? now - L.act_mark_ns : 0;
  const uint64_t marked_raw = L.occ_mark_acc + inflight;
  const uint64_t marked = marked_raw > L.occ_credit ? marked_raw - L.occ_credit : 0;
  const uint64_t unt = L.untracked_ns.load(std::memory_order_relaxed);
  const bool skip = unt && unt + 2 * period >= L.occ_window_start;
  // Charge what the samples saw beyond the markers' share, less a tolerance
  // for sampling error (one period either way, 10 %).
  const uint64_t seen = L.occ_busy_acc;
  const uint64_t slack = period + marked / 10;
  if (!skip && seen > marked + slack) {
    const uint64_t extra = seen - marked - slack;
    // Processor sharing as for marker charges: k pods busy at once pay 1/k each
    // (the board's virtual time is tied to marker intervals, so scale directly).
    const int k = L.board ? std::max(1, (int)__atomic_load_n(&L.board->n_active, __ATOMIC_RELAXED)) : 1;
    const uint64_t charge = extra / (uint64_t)k;
    charge_tokens(L, (int64_t)charge);
    L.win_charge += charge;
    L.charged_total.fetch_add(charge, std::memory_order_relaxed);
    L.occ_extra_total.fetch_add(charge, std::memory_order_relaxed);
    trace_emit(VGPU_EV_GPU_TIME, dev, charge, extra);
  }
  L.occ_busy_acc = L.occ_mark_acc = 0;
  L.occ_credit = inflight;
  L.occ_window_start = now;
}

void limiter_main() {
  g_thread_alive.store(1);
  // Our polling must not be refused (or break) an application's graph capture
  // in hipStreamCaptureModeGlobal on another thread.
  if (auto xm = REAL_HIP(hipThreadExchangeStreamCaptureMode)) {
    hipStreamCaptureMode m = hipStreamCaptureModeRelaxed;
    (void)xm(&m);
  }
  uint64_t last = mono_ns(), last_mask = last, last_pool = last, last_auto = last;
  uint64_t mask_sig = 0;
  State& s = st();
  while (!g_shutdown.load(std::memory_order_relaxed)) {
    bool busy = false;
    if (g_throttle_any.load(std::memory_order_relaxed))
      for (int d = 0; d < VGPU_MAX_DEVICES; ++d) {
        DevLimiter& L = g_lim[d];
        if (!L.active) continue;
        L.idle.store(0, std::memory_order_relaxed);
        busy |= reap(d, L);
        // reap published idleness: a marker pushed meanwhile is picked up now
        if (!busy && L.idle.load(std::memory_order_seq_cst) && rings_pending(L)) busy = true;
      }
    if (busy) {
      sleep_ns(100000);  // 100 µs: completion-time resolution while work is in flight
    } else {
      std::unique_lock<std::mutex> lk(g_cv_mu);
      g_cv.wait_for(lk, std::chrono::milliseconds(2));
    }
    const uint64_t now = mono_ns();
    const double dt = (double)(now - last);
    last = now;
    for (int d = 0; d < VGPU_MAX_DEVICES; ++d) {
      DevLimiter& L = g_lim[d];
      if (!L.active) {
        // a spatial auto member is not throttled, but its CU claim lives only
        // as long as its board slot stays fresh
        if (L.auto_share && L.board) board_heartbeat(L.board, L.board_slot);
        continue;
      }
      // Credit rate.  force: the hard cap (limit % of wall time).  default:
      // work-conserving weighted fair share among the pods of this GPU that
      // have work outstanding (board entitlement) -- a pod alone is not held
      // back, k equal pods get 1/k each, a 25 % and a 75 % pod get 1:3 --
      // the reference's "throttle only under contention" made proportional.
      double rate = L.frac;
      if (s.lim.core_policy != 1 && L.board) rate = fmax(L.frac, board_entitlement(L.board, L.board_slot));
      const int64_t add = (int64_t)(rate * dt);
      int64_t cur = L.tokens.load(std::memory_order_relaxed), nv;
      do {
        nv = cur + add;
        if (nv > L.cap) nv = L.cap;
      } while (!L.tokens.compare_exchange_weak(cur, nv, std::memory_order_relaxed));
      if (L.board) board_heartbeat(L.board, L.board_slot);
      occ_step(d, L, now);
      // Publish this process's fair-share utilization of the last ~120 ms window
      // (the reference watcher's cadence) for the monitor's metrics.
      if (now - L.win_start >= 120000000ull) {
        const double win = (double)(now - L.win_start);
        if (s.region) {
          __atomic_store_n(&s.region->dev[d].busy_permille,
                           (uint32_t)fmin(1000.0, 1000.0 * L.win_charge / win), __ATOMIC_RELAXED);
          __atomic_store_n(&s.region->dev[d].busy_ns, now, __ATOMIC_RELEASE);
        }
        VLOG_DEBUG("limiter dev %d: charged %.1f%% busy %.1f%% of %.0f ms (target %.0f%%, tokens %.2f ms)",
                   d, 100.0 * L.win_charge / win, 100.0 * L.win_busy / win, win / 1e6, 100 * L.frac,
                   L.tokens.load() / 1e6);
        L.win_charge = L.win_busy = 0;
        L.win_start = now;
      }
    }
    if (g_auto_any.load(std::memory_order_relaxed) && now - last_auto >= 50000000ull) {
      last_auto = now;
      auto_step();
    }
    // Stream-ordered pools give memory back on their own (release threshold):
    // keep their charge current.
    if (now - last_pool >= 50000000ull) {
      last_pool = now;
      if (pools_any()) pools_sync(false);
      for (int d = 0; d < VGPU_MAX_DEVICES; ++d) mem_sync_runtime(d);
    }
    // Re-apply CU masks when the region's masks change (elastic resizing by
    // the node monitor / device plugin).
    if (s.region && now - last_mask >= 10000000ull) {
      last_mask = now;
      uint64_t sig = 1469598103934665603ull;
      for (int d = 0; d < VGPU_MAX_DEVICES; ++d)
        for (int w = 0; w < VGPU_CU_MASK_WORDS; ++w)
          sig = (sig ^ __atomic_load_n(&s.region->dev[d].cu_mask[w], __ATOMIC_RELAXED)) *
                1099511628211ull;
      if (sig != mask_sig) {
        if (mask_sig != 0) cumask_reapply_all();
        mask_sig = sig;
        configure();
      }
    }
  }
  g_thread_alive.store(0);
}

void priority_gate(vgpu_shared_region_t* r) {
  // Monitor preemption: a higher-priority task is active on the device.
  if (__builtin_expect(__atomic_load_n(&r->recent_kernel, __ATOMIC_RELAXED) >= 0, 1)) {
    if (__atomic_load_n(&r->recent_kernel, __ATOMIC_RELAXED) != 2)
      __atomic_store_n(&r->recent_kernel, 2, __ATOMIC_RELAXED);
    return;
  }
  uint64_t t0 = mono_ns();
  while (__atomic_load_n(&r->recent_kernel, __ATOMIC_RELAXED) < 0) sleep_ns(1000000);
  const uint64_t waited = mono_ns() - t0;
  if (vgpu_proc_slot_t* sl = my_slot())
    __atomic_fetch_add(&sl->throttle_wait_ns, waited, __ATOMIC_RELAXED);
  trace_emit(VGPU_EV_PRIORITY_BLOCK, -1, waited, 0);
  __atomic_store_n(&r->recent_kernel, 2, __ATOMIC_RELAXED);
}

// A launch the markers deliberately do not charge (cross-check skips its window).
void note_untracked(DevLimiter& L) {
  const uint64_t now = mono_ns();
  if (now - L.untracked_ns.load(std::memory_order_relaxed) > 1000000ull)
    L.untracked_ns.store(now, std::memory_order_relaxed);
}

}  // namespace

// Collective kernels (RCCL) are never held by the temporal limiter (they are
// still charged): every rank's kernel must be resident for a collective to
// progress, so holding one rank's launch mid-step stalls the others (distributed backend row;
// §7.4 item 8).  A kernel is RCCL's when its host stub lives in librccl (or a
// library matching VGPU_THROTTLE_EXEMPT).  Decided once per function pointer
// and launching thread: the cache is thread-local, so a throttled launch takes
// no lock here (multi-threaded launchers never serialise on it).
bool exempt_kernel(const void* fn) {
  if (!fn) return false;
  thread_local const void* last_fn = nullptr;
  thread_local bool last_ex = false;
  if (fn == last_fn) return last_ex;
  thread_local std::unordered_map<const void*, bool> cache;
  auto it = cache.find(fn);
  if (it != cache.end()) {
    last_fn = fn;
    return last_ex = it->second;
  }
  bool ex = false;
  Dl_info di;
  if (dladdr(fn, &di) && di.dli_fname) {
    const char* extra = env_first("VGPU_THROTTLE_EXEMPT");
    ex = strstr(di.dli_fname, "rccl") || strstr(di.dli_fname, "nccl") ||
         (extra && *extra && strstr(di.dli_fname, extra));
  }
  cache.emplace(fn, ex);
  last_fn = fn;
  return last_ex = ex;
}

// Publish the calling thread's batched launch counts now (synchronize hooks:
// a caller that waited for its work reads current slot counters).
void limiter_flush_thread() {
  if (tl_counts.since) flush_counts(tl_counts, mono_ns());
}

void limiter_start() {
  configure();
  int expected = 0;
  if (!g_thread_running.compare_exchange_strong(expected, 1)) return;
  State& s = st();
  bool need = g_throttle_any.load() || (s.region && s.region->num_devices > 0);
  if (!need) return;
  std::thread(limiter_main).detach();
}

void limiter_stop() {
  g_shutdown.store(1);
  g_cv.notify_all();
  for (int i = 0; i < 200 && g_thread_alive.load(); ++i) sleep_ns(1000000);
  if (tl_counts.since) flush_counts(tl_counts, mono_ns());
  for (auto& L : g_lim)
    if (L.board) {
      board_release(L.board, L.board_slot);
      L.board = nullptr;
    }
}

void limiter_after_fork() {
  // The child has no limiter thread and no live markers of its own.
  g_thread_running.store(0);
  g_thread_alive.store(0);
  g_track_gen.fetch_add(1);
  tl_counts = ThreadCounts{};
  for (auto& L : g_lim) {
    L.tracks.clear();  // the parent's rings (leaked in the child; their events belong to the parent)
    L.inflight_pub.store(0);
    L.busy.store(0);
    L.idle.store(1);
    L.board = nullptr;
    L.board_slot = -1;
    L.board_tried = false;
    L.board_ready.store(0);
  }
}

// `collective`: the launch is a collective's (never held, always charged).
bool limiter_on_launch(int dev, uint64_t wg, const void* fn, uint32_t kernels, bool collective) {
  State& s = st();
  if (!s.enabled) return false;
  suspend_gate();
  if (s.region) priority_gate(s.region);
  ThreadCounts& c = tl_counts;
  ++c.launches;
  const bool ok_dev = dev >= 0 && dev < VGPU_MAX_DEVICES;
  if (g_auto_any.load(std::memory_order_relaxed) && ok_dev && g_lim[dev].auto_share)
    ++c.kern[dev];  // progress: one step of a graph replay, or one kernel
  // Batched: the slot counters and the auto policy's count are shared lines.
  if (++c.since >= 64) flush_counts(c, mono_ns());
  else if (c.since == 1) {
    const uint64_t now = mono_ns();
    if (now - c.last_flush_ns > 1000000ull) flush_counts(c, now);  // an idle thread's first launch: current
  }
  (void)kernels;
  const bool throttling = g_throttle_any.load(std::memory_order_relaxed) != 0;
  if (__builtin_expect(!throttling && !trace_on(), 1)) return false;
  const bool exempt = throttling && (collective || exempt_kernel(fn));
  trace_emit(VGPU_EV_LAUNCH, dev, wg, exempt ? 1 : 0);
  if (!throttling || !ok_dev) return false;
  DevLimiter& L = g_lim[dev];
  if (!L.active) return false;
  if (__builtin_expect(L.pool_scale_pending.load(std::memory_order_relaxed), 0)) apply_pool_scale(dev, L);
  if (s.region && s.lim.core_policy != 1 &&
      __atomic_load_n(&s.region->utilization_switch, __ATOMIC_RELAXED) == 0) {
    note_untracked(L);
    return false;  // monitor says no contention: run unthrottled
  }
  // An eager collective kernel is never held (its peers would wait on it) but
  // is charged like any launch: its marker's GPU time is paid by the next
  // held launch of the pod (an exemption from the charge let a
  // pod's collective time escape its cap).
  if (exempt) return true;
  // VGPU_LIMITER_DRYRUN=1: measure and charge, never wait (diagnostics).
  static const bool dryrun = env_bool(env_first("VGPU_LIMITER_DRYRUN"), false);
  if (dryrun) return true;
  vgpu_proc_slot_t* sl = my_slot();
  if (L.max_running > 0 && g_open_captures.load(std::memory_order_acquire) == 0) {
    if (!L.board_tried) {
      std::lock_guard<std::mutex> g(L.mu);
      attach_board(dev, L);
    }
    if (L.board) {
      uint64_t g0 = 0;
      while (!board_gate(L.board, L.board_slot, L.max_running, L.run_quantum_ns)) {
        if (!g0) g0 = mono_ns();
        sleep_ns(100000);  // 0.1 ms
        if (g_shutdown.load(std::memory_order_relaxed)) break;
      }
      if (g0) {
        const uint64_t waited = mono_ns() - g0;
        if (sl) __atomic_fetch_add(&sl->throttle_wait_ns, waited, __ATOMIC_RELAXED);
        trace_emit(VGPU_EV_THROTTLE, dev, waited, wg);
      }
    }
  }
  // Wait while the bucket cannot pay for the work already in flight; once
  // overdrawn, hold until it has refilled by a whole quantum.  In flight: the
  // launches the last drain saw uncharged, plus this thread's since then.
  uint64_t t0 = 0;
  for (;;) {
    // Until the first marker completes, assume 1 ms per launch in flight.
    int64_t per = L.ema_charge.load(std::memory_order_relaxed);
    if (per <= 0) per = 1000000;
    const int64_t pending = (L.inflight_pub.load(std::memory_order_relaxed) + own_unpublished(dev)) * per;
    const int64_t avail = L.tokens.load(std::memory_order_relaxed) - pending;
    if (L.hold.load(std::memory_order_relaxed)) {
      if (avail >= L.quantum) {
        L.hold.store(0, std::memory_order_relaxed);
        break;
      }
    } else if (avail >= 0) {
      break;
    } else {
      L.hold.store(1, std::memory_order_relaxed);
    }
    if (!t0) t0 = mono_ns();
    sleep_ns(200000);  // 0.2 ms
    if (g_shutdown.load(std::memory_order_relaxed)) break;
  }
  if (t0) {
    const uint64_t waited = mono_ns() - t0;
    if (sl) __atomic_fetch_add(&sl->throttle_wait_ns, waited, __ATOMIC_RELAXED);
    trace_emit(VGPU_EV_THROTTLE, dev, waited, wg);
  }
  return true;
}

// After a tracked launch: record a marker on its stream and push it onto this
// thread's ring.  Lock-free; the only shared write is a wake-up of the limiter
// thread when it has gone idle.
void limiter_track(int dev, hipStream_t stream, hipError_t launch_rc, uint64_t submit_ns) {
  if (dev < 0 || dev >= VGPU_MAX_DEVICES) return;
  DevLimiter& L = g_lim[dev];
  // Not tracked: the launch failed, or it was captured into a graph (it runs
  // when the graph is launched, and is charged then).  A concurrency-gate turn
  // taken for it must not stay claimed with nothing to drain it.
  auto untracked = [&] {
    if (L.max_running > 0 && L.board && !L.busy.load(std::memory_order_relaxed) && !rings_pending(L))
      board_gate_abort(L.board, L.board_slot);
  };
  if (launch_rc != hipSuccess || stream_capturing(stream)) return untracked();
  if (__builtin_expect(!L.board_ready.load(std::memory_order_acquire), 0)) {
    std::lock_guard<std::mutex> g(L.mu);  // once per device: join the GPU's share board now
    attach_board(dev, L);
    L.board_ready.store(1, std::memory_order_release);
  }
  Track* t = my_track(dev);
  const uint32_t h = t->head.load(std::memory_order_relaxed);
  // Ring full (kRing markers of this thread in flight): the launch runs
  // inside the busy interval those markers keep open, and is not counted in
  // flight (an uncovered launch would never be retired and would hold the
  // bucket's quantum check forever).
  if (h - t->tail.load(std::memory_order_acquire) >= kRing) return;
  hipEvent_t ev = t->spare;
  t->spare = nullptr;
  if (!ev) {
    const uint32_t ft = t->ftail.load(std::memory_order_relaxed);
    if (ft != t->fhead.load(std::memory_order_acquire)) {
      ev = t->fring[ft & kMask];
      t->ftail.store(ft + 1, std::memory_order_release);
    } else if (REAL_HIP(hipEventCreateWithFlags)(&ev, hipEventDisableTiming) != hipSuccess) {
      return untracked();
    }
  }
  if (REAL_HIP(hipEventRecord)(ev, stream) != hipSuccess) {
    t->spare = ev;
    return untracked();
  }
  t->ring[h & kMask] = Marker{ev, submit_ns ? submit_ns : mono_ns(), stream, 1};
  t->launches.store(t->launches.load(std::memory_order_relaxed) + 1, std::memory_order_relaxed);
  t->head.store(h + 1, std::memory_order_release);
  // Wake the limiter thread if it went idle (see reap: it re-checks the rings
  // after publishing idleness, so a push that misses the flag is not lost).
  std::atomic_thread_fence(std::memory_order_seq_cst);
  if (L.idle.load(std::memory_order_relaxed) && L.idle.exchange(0, std::memory_order_relaxed)) g_cv.notify_one();
}

// What the compute-share policy of `dev` is doing (bench / tests):
// out[0] auto phase of the GPU's share board (-1: not an auto member / no board),
// out[1] busy members the board's decision was made for, out[2] 1 when the
// board holds a decision for that member count, out[3] 1 while this process
// runs on CUs of its own, out[4] CUs in the region's mask (0 = every CU),
// out[5] 1 while the temporal limiter is active for the device, out[6] ns this
// process has waited in the limiter, out[7] ns charged on KFD occupancy
// evidence beyond the markers (occ_step).
void limiter_share_state(int dev, int64_t out[8]) {
  for (int i = 0; i < 8; ++i) out[i] = 0;
  out[0] = -1;
  if (dev < 0 || dev >= VGPU_MAX_DEVICES) return;
  DevLimiter& L = g_lim[dev];
  if (L.auto_share && L.board) {
    vgpu_board_t* b = L.board;
    out[0] = __atomic_load_n(&b->auto_phase, __ATOMIC_ACQUIRE);
    const int n = __atomic_load_n(&b->auto_members, __ATOMIC_RELAXED);
    out[1] = n;
    out[2] = n > 0 && n < VGPU_AUTO_MEMO && __atomic_load_n(&b->auto_memo_ns[n], __ATOMIC_RELAXED) != 0;
  }
  out[3] = L.spatial;
  State& s = st();
  if (s.region)
    for (int w = 0; w < VGPU_CU_MASK_WORDS; ++w)
      out[4] += __builtin_popcountll(__atomic_load_n(&s.region->dev[dev].cu_mask[w], __ATOMIC_RELAXED));
  out[5] = L.active ? 1 : 0;
  if (vgpu_proc_slot_t* sl = my_slot()) out[6] = (int64_t)__atomic_load_n(&sl->throttle_wait_ns, __ATOMIC_RELAXED);
  out[7] = (int64_t)L.occ_extra_total.load(std::memory_order_relaxed);
}

// Fair-share GPU ns charged / wall ns busy so far on `dev` (tests, metrics).
void limiter_stats(int dev, uint64_t* charged, uint64_t* busy) {
  if (dev < 0 || dev >= VGPU_MAX_DEVICES) return;
  if (charged) *charged = g_lim[dev].charged_total.load();
  if (busy) *busy = g_lim[dev].busy_total.load();
}

}  // namespace vgpu
