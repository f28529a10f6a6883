// Lazy initialisation, fork handling, exit cleanup and suspend/resume signals.
//
// Reference behaviour: libvgpu.so cuInit → pthread_once(preInit) → postInit
// (allocator_init, set_task_pid, init_utilization_watcher), exit_handler, and
// SIGUSR2/SIGUSR1 → sig_swap_stub / sig_restore_stub.
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>

#include "common.h"
#include "state.h"

namespace vgpu {

static State* g_state = nullptr;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

State& st() {
  if (__builtin_expect(g_state == nullptr, 0)) {
    // Leaked on purpose: hooks may run during static destruction.
    static State* s = new State();
    g_state = s;
  }
  return *g_state;
}

static void on_exit_release() {
  limiter_stop();
  vmem_stop();
  State& s = st();
  if (s.region && s.slot >= 0) {
    region_release_slot(s.region, s.slot);
    s.slot = -1;
  }
}

static void sig_suspend(int) {
  State& s = st();
  s.suspended.store(1, std::memory_order_relaxed);
  if (vgpu_proc_slot_t* sl = my_slot())
    __atomic_store_n(&sl->status, VGPU_PROC_SUSPENDED, __ATOMIC_RELAXED);
}

static void sig_resume(int) {
  State& s = st();
  s.suspended.store(0, std::memory_order_relaxed);
  if (vgpu_proc_slot_t* sl = my_slot())
    __atomic_store_n(&sl->status, VGPU_PROC_RUNNING, __ATOMIC_RELAXED);
}

static void install_signal(int sig, void (*fn)(int)) {
  struct sigaction old;
  if (sigaction(sig, nullptr, &old) == 0 && old.sa_handler != SIG_DFL && old.sa_handler != SIG_IGN)
    return;  // the application owns this signal; leave it alone
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_handler = fn;
  sa.sa_flags = SA_RESTART;
  sigaction(sig, &sa, nullptr);
}

// VGPU_CRASH_TRACE=1: on SIGSEGV / SIGBUS / SIGABRT print the native stack
// (module + offset per frame, for addr2line against the same build) to stderr,
// then die as the signal would have.  Diagnostics only; async-signal-safe calls.
static void crash_trace(int sig, siginfo_t* info, void*) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  char line[160];
  const int k = snprintf(line, sizeof line, "[vgpu] signal %d at address %p, native stack:\n", sig,
                         info ? info->si_addr : nullptr);
  if (k > 0) (void)!write(2, line, (size_t)k);
  for (int i = 0; i < n; ++i) {
    Dl_info di;
    int m;
    if (dladdr(frames[i], &di) && di.dli_fname)
      m = snprintf(line, sizeof line, "  #%d %s+0x%lx %s\n", i, di.dli_fname,
                   (unsigned long)((char*)frames[i] - (char*)di.dli_fbase), di.dli_sname ? di.dli_sname : "");
    else
      m = snprintf(line, sizeof line, "  #%d %p\n", i, frames[i]);
    if (m > 0) (void)!write(2, line, (size_t)m);
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

static void install_crash_trace() {
  if (!env_bool(env_first("VGPU_CRASH_TRACE"), false)) return;
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = crash_trace;
  sa.sa_flags = SA_SIGINFO | SA_RESETHAND;
  for (int sig : {SIGSEGV, SIGBUS, SIGABRT}) sigaction(sig, &sa, nullptr);
}

static void atfork_child() {
  // The child inherits the parent's mapping but not its slot; it claims its
  // own slot lazily on first use.
  State& s = st();
  s.slot = -1;
  s.pid = getpid();
  hostpid_after_fork();
  limiter_after_fork();
  vmem_after_fork();
  vmm_after_fork();
  pools_after_fork();
  if (s.region) {
    s.slot = region_claim_slot(s.region, s.pid, self_host_pid(nullptr), s.lim.priority);
    hostpid_publish();
  }
  {
    std::lock_guard<std::mutex> g(s.ledger_mu);
    s.ledger.clear();
  }
  for (auto& t : s.dev_touched) t.store(0);
  mem_after_fork();
  trace_after_fork();
}

static void do_init() {
  State& s = st();
  s.pid = getpid();
  bool disabled = env_bool(env_first("VGPU_DISABLE_CONTROL", "CUDA_DISABLE_CONTROL"), false);
  s.lim = limits_from_env();
  s.report_masked_cus = env_bool(env_first("VGPU_REPORT_MASKED_CUS"), false);
  s.active_oom_killer = env_bool(env_first("ACTIVE_OOM_KILLER"), false);
  s.context_charge = parse_mem(env_first("VGPU_CONTEXT_CHARGE"));
  s.ctx_measure = env_bool(env_first("VGPU_CONTEXT_MEASURE"), true);
  s.ctx_max = parse_mem(env_first("VGPU_CONTEXT_MAX"));
  if (!s.ctx_max) s.ctx_max = 4ull << 30;
  for (auto& f : s.kfd_vram_fd) f.store(-2);
  install_crash_trace();  // diagnostics work with control disabled too
  s.enabled = !disabled;
  if (!s.enabled) {
    VLOG_INFO("vgpu control disabled by environment");
    s.init_done.store(1, std::memory_order_release);
    return;
  }
  const char* path = env_first("VGPU_SHARED_REGION", "CUDA_DEVICE_MEMORY_SHARED_CACHE");
  s.region = region_map(path, &s.lim, &s.region_fd);
  if (!s.region && path) {
    VLOG_WARN("falling back to a private region (could not map %s)", path);
    s.region = region_map(nullptr, &s.lim, &s.region_fd);
  }
  if (s.region) {
    s.slot = region_claim_slot(s.region, s.pid, self_host_pid(nullptr), s.lim.priority);
    if (s.slot < 0) VLOG_ERR("no free process slot in the shared region");
    hostpid_publish();
  }
  trace_open();
  install_signal(SIGUSR2, sig_suspend);
  install_signal(SIGUSR1, sig_resume);
  atexit(on_exit_release);
  pthread_atfork(nullptr, nullptr, atfork_child);
  for (int i = 0; i < s.lim.num_devices; ++i) {
    if (s.lim.mem_limit[i] || s.lim.cu_limit[i])
      VLOG_INFO("device %d: memory limit %llu MiB, cu limit %u%%", i,
                (unsigned long long)(s.lim.mem_limit[i] >> 20), s.lim.cu_limit[i]);
  }
  limiter_start();
  s.init_done.store(1, std::memory_order_release);
}

void ensure_init() {
  if (__builtin_expect(st().init_done.load(std::memory_order_acquire), 1)) return;
  pthread_once(&g_once, do_init);
}

void suspend_gate() {
  State& s = st();
  auto held = [&] {
    return s.suspended.load(std::memory_order_relaxed) || s.vmm_evicted.load(std::memory_order_relaxed);
  };
  if (__builtin_expect(!held(), 1)) return;
  // Inside a HookScope that passed the gate already: the evict thread waits for
  // this call to finish, so waiting here would deadlock with it.
  if (vmm_in_scope()) return;
  uint64_t t0 = mono_ns();
  while (held()) sleep_ns(1000000);  // 1 ms
  const uint64_t waited = mono_ns() - t0;
  if (vgpu_proc_slot_t* sl = my_slot())
    __atomic_fetch_add(&sl->throttle_wait_ns, waited, __ATOMIC_RELAXED);
  trace_emit(VGPU_EV_SUSPEND, -1, waited, 0);
}

}  // namespace vgpu
