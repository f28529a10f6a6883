// Compute-share enforcement on the dispatch path.
//
// Reference behaviour: libvgpu.so's
// `utilization_watcher` thread samples per-process SM utilization every 120 ms
// and feeds a global token counter; `rate_limiter(grids, blocks)` runs on
// every cuLaunchKernel: it blocks while the monitor has set recent_kernel < 0
// (priority preemption), sets recent_kernel = 2, returns when the limit is 0 or
// >= 100 or utilizationSwitch == 0, and otherwise CAS-decrements the counter
// by `grids`, sleeping while it is negative.
//
// MI355X design: the PRIMARY mechanism is spatial (XCD-balanced CU masks on
// every HSA queue, cumask.cpp) which is exact and costs nothing per dispatch.
// This temporal limiter only engages when a mask cannot express the share
// (GPU_CORE_UTILIZATION_POLICY=force, or no mask) — it is a workgroup-rate
// token bucket whose refill rate is adapted so that the sampled utilization
// tracks the limit (multiplicative controller), rather than a fixed
// SM²-proportional step.
#include <dirent.h>
#include <dlfcn.h>
#include <math.h>

#include <unordered_map>

#include <thread>

#include "common.h"
#include "state.h"

namespace vgpu {

thread_local int tl_device = 0;
thread_local int tl_in_hip_alloc = 0;

struct DevLimiter {
  std::atomic<int64_t> tokens{0};
  std::atomic<uint64_t> launched{0};  // workgroups launched (for rate estimation)
  std::atomic<uint64_t> waited{0};    // launches that had to wait
  double rate = 0;                    // workgroups / second
  double cap = 0;                     // bucket depth (workgroups)
  int active = 0;                     // temporal throttling enabled for this device
  double util_acc = 0;
  int util_n = 0;
};

static DevLimiter g_lim[VGPU_MAX_DEVICES];
static std::atomic<int> g_throttle_any{0};
static std::atomic<int> g_watcher_running{0};

// Utilization sampling -------------------------------------------------------------
// Returns percent busy of device `dev` attributable to this container, or -1.
extern int cumask_device_cus(int dev);        // CUs available to us (mask or physical)
extern uint32_t cumask_driver_uid(int dev);   // KFD gpu_id of device, 0 = unknown

static double sample_fake(int dev) {
  const char* f = getenv("VGPU_FAKE_UTIL_FILE");
  if (!f) return -1;
  FILE* fp = fopen(f, "r");
  if (!fp) return -1;
  int d;
  double u;
  double out = -1;
  while (fscanf(fp, "%d %lf", &d, &u) == 2)
    if (d == dev) out = u;
  fclose(fp);
  return out;
}

static double sample_kfd(int dev) {
  State& s = st();
  if (!s.region) return -1;
  uint32_t uid = cumask_driver_uid(dev);
  int cus = cumask_device_cus(dev);
  if (cus <= 0) return -1;
  double busy = 0;
  bool any = false;
  for (int i = 0; i < VGPU_MAX_PROCS; ++i) {
    const vgpu_proc_slot_t& sl = s.region->procs[i];
    if (sl.status == VGPU_PROC_FREE) continue;
    int pid = sl.host_pid > 0 ? sl.host_pid : sl.pid;
    char dir[128];
    snprintf(dir, sizeof dir, "/sys/class/kfd/kfd/proc/%d", pid);
    DIR* d = opendir(dir);
    if (!d) continue;
    struct dirent* e;
    while ((e = readdir(d))) {
      if (strncmp(e->d_name, "stats_", 6)) continue;
      if (uid && (uint32_t)strtoul(e->d_name + 6, nullptr, 10) != uid) continue;
      char path[512];
      snprintf(path, sizeof path, "%s/%s/cu_occupancy", dir, e->d_name);
      FILE* fp = fopen(path, "r");
      if (!fp) continue;
      int v = 0;
      if (fscanf(fp, "%d", &v) == 1) { busy += v; any = true; }
      fclose(fp);
    }
    closedir(d);
  }
  if (!any) return -1;
  double u = 100.0 * busy / cus;
  return u > 100 ? 100 : u;
}

static double sample_util(int dev) {
  double u = sample_fake(dev);
  if (u >= 0) return u;
  return sample_kfd(dev);
}

// Decide per device whether temporal throttling applies.
static void configure() {
  State& s = st();
  int any = 0;
  for (int d = 0; d < VGPU_MAX_DEVICES; ++d) {
    uint32_t lim = s.region ? s.region->dev[d].cu_limit : s.lim.cu_limit[d];
    bool has_mask = false;
    if (s.region)
      for (int w = 0; w < VGPU_CU_MASK_WORDS; ++w) has_mask |= s.region->dev[d].cu_mask[w] != 0;
    bool want = lim > 0 && lim < 100 && s.lim.core_policy != 2;
    // A CU mask already enforces the share spatially; temporal limiting on top
    // of it only when explicitly forced.
    if (has_mask && s.lim.core_policy != 1) want = false;
    if (!has_mask && s.lim.core_policy == 0 &&
        env_bool(env_first("VGPU_CU_MASK_FROM_LIMIT"), true))
      want = false;  // cumask.cpp derives a balanced mask from the limit
    g_lim[d].active = want;
    any |= want;
  }
  g_throttle_any.store(any, std::memory_order_release);
}

static void watcher_main() {
  const uint64_t tick_ns =
      (uint64_t)(1e6 * (getenv("VGPU_LIMITER_TICK_MS") ? atof(getenv("VGPU_LIMITER_TICK_MS")) : 10.0));
  const uint64_t window_ns = 120000000ull;  // 120 ms control window (reference cadence)
  uint64_t last = mono_ns(), last_ctl = last;
  uint64_t seen_seq = 0;
  uint64_t mask_sig = 0;
  State& s = st();
  for (;;) {
    sleep_ns(tick_ns);
    uint64_t now = mono_ns();
    double dt = (now - last) * 1e-9;
    last = now;
    // Re-apply CU masks when the region's masks change (elastic resizing by
    // the node monitor / device plugin).
    if (s.region) {
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
      (void)seen_seq;
    }
    if (!g_throttle_any.load(std::memory_order_relaxed)) continue;
    for (int d = 0; d < VGPU_MAX_DEVICES; ++d) {
      DevLimiter& L = g_lim[d];
      if (!L.active) continue;
      if (L.rate > 0) {
        int64_t add = (int64_t)(L.rate * dt);
        int64_t cur = L.tokens.load(std::memory_order_relaxed);
        int64_t nv;
        do {
          nv = cur + add;
          if (nv > (int64_t)L.cap) nv = (int64_t)L.cap;
        } while (!L.tokens.compare_exchange_weak(cur, nv, std::memory_order_relaxed));
      }
      double u = sample_util(d);
      if (u >= 0) { L.util_acc += u; L.util_n++; }
    }
    if (now - last_ctl < window_ns) continue;
    double wdt = (now - last_ctl) * 1e-9;
    last_ctl = now;
    for (int d = 0; d < VGPU_MAX_DEVICES; ++d) {
      DevLimiter& L = g_lim[d];
      if (!L.active) continue;
      uint32_t lim = s.region ? s.region->dev[d].cu_limit : s.lim.cu_limit[d];
      uint64_t launched = L.launched.exchange(0);
      uint64_t waited = L.waited.exchange(0);
      double obs_rate = launched / wdt;
      if (L.util_n == 0) continue;  // no utilization signal: keep the current rate
      double u = L.util_acc / L.util_n;
      L.util_acc = 0;
      L.util_n = 0;
      double target = (double)lim;
      if (L.rate <= 0) {
        // First window: calibrate from what the application actually issued.
        L.rate = obs_rate > 0 ? obs_rate * fmin(1.0, target / fmax(u, 1.0)) : 0;
      } else {
        double ratio = (target + 1.0) / (u + 1.0);
        ratio = fmax(0.5, fmin(2.0, ratio));
        // Only grow the grant when the application was actually held back.
        if (ratio > 1.0 && waited == 0) ratio = 1.0;
        L.rate = fmax(L.rate * ratio, 64.0);
      }
      L.cap = fmax(L.rate * 0.05, 1024.0);  // 50 ms of burst
      VLOG_DEBUG("limiter dev %d: util %.1f%% target %u%% rate %.0f wg/s (obs %.0f)", d, u, lim,
                 L.rate, obs_rate);
    }
  }
}

void limiter_start() {
  configure();
  int expected = 0;
  if (!g_watcher_running.compare_exchange_strong(expected, 1)) return;
  State& s = st();
  bool need = g_throttle_any.load() || (s.region && s.region->num_devices > 0);
  if (!need) return;
  std::thread(watcher_main).detach();
}

static void priority_gate(vgpu_shared_region_t* r) {
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

// Collective kernels (RCCL) are exempt from the temporal limiter: every rank's
// kernel must be resident for a collective to progress, so throttling one
// rank's launches stalls the others (distributed backend row;
// §7.4 item 8).  A kernel is RCCL's when its host stub lives in librccl (or a
// library matching VGPU_THROTTLE_EXEMPT).  Decided once per function pointer.
static bool exempt_kernel(const void* fn) {
  if (!fn) return false;
  static std::mutex mu;
  static std::unordered_map<const void*, bool> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(fn);
  if (it != cache.end()) return it->second;
  bool ex = false;
  Dl_info di;
  if (dladdr(fn, &di) && di.dli_fname) {
    const char* extra = env_first("VGPU_THROTTLE_EXEMPT");
    ex = strstr(di.dli_fname, "rccl") || strstr(di.dli_fname, "nccl") ||
         (extra && *extra && strstr(di.dli_fname, extra));
  }
  cache.emplace(fn, ex);
  return ex;
}

void limiter_on_launch(int dev, uint64_t wg, const void* fn) {
  State& s = st();
  if (!s.enabled) return;
  suspend_gate();
  vgpu_proc_slot_t* sl = my_slot();
  if (s.region) priority_gate(s.region);
  if (sl) __atomic_fetch_add(&sl->launches, 1, __ATOMIC_RELAXED);
  const bool throttling = g_throttle_any.load(std::memory_order_relaxed) != 0;
  if (__builtin_expect(!throttling && !trace_on(), 1)) return;
  const bool exempt = throttling && exempt_kernel(fn);
  trace_emit(VGPU_EV_LAUNCH, dev, wg, exempt ? 1 : 0);
  if (!throttling || exempt) return;
  if (dev < 0 || dev >= VGPU_MAX_DEVICES) return;
  DevLimiter& L = g_lim[dev];
  if (!L.active) return;
  L.launched.fetch_add(wg, std::memory_order_relaxed);
  if (s.region && s.lim.core_policy != 1 &&
      __atomic_load_n(&s.region->utilization_switch, __ATOMIC_RELAXED) == 0)
    return;  // monitor says no contention: run unthrottled
  if (L.rate <= 0) return;  // not calibrated yet
  int64_t cur = L.tokens.load(std::memory_order_relaxed);
  uint64_t t0 = 0;
  for (;;) {
    if (cur > 0) {
      if (L.tokens.compare_exchange_weak(cur, cur - (int64_t)wg, std::memory_order_relaxed)) break;
      continue;
    }
    if (!t0) {
      t0 = mono_ns();
      L.waited.fetch_add(1, std::memory_order_relaxed);
    }
    sleep_ns(500000);  // 0.5 ms
    cur = L.tokens.load(std::memory_order_relaxed);
  }
  if (t0) {
    const uint64_t waited = mono_ns() - t0;
    if (sl) __atomic_fetch_add(&sl->throttle_wait_ns, waited, __ATOMIC_RELAXED);
    trace_emit(VGPU_EV_THROTTLE, dev, waited, wg);
  }
}

}  // namespace vgpu
