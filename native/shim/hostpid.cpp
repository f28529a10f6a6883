// Host-PID resolution for a process inside a pod's PID namespace.
//
// Reference behaviour: libvgpu.so `set_task_pid` (3373 B) takes the node-wide
// unified lock (/tmp/vgpulock/lock, mounted by the device plugin at
// pkg/device-plugin/nvidiadevice/nvinternal/plugin/server.go:357-369), lists
// the device's processes through NVML, creates the CUDA context, lists them
// again and takes the new entry as its host pid.
//
// ROCm design: the per-process KFD sysfs directory
// /sys/class/kfd/kfd/proc/<host pid> is created synchronously inside the
// first open("/dev/kfd") of a process, and sysfs is not PID-namespaced.  The
// shim interposes open/open64 (libhsa-runtime64 imports open@GLIBC_2.2.5) and
// brackets exactly that one call: flock(unified lock) → list KFD entries →
// real open → list again → unlock.  The bracket is microseconds wide, so the
// diff has one entry unless a process outside our lock opened /dev/kfd in the
// same instant; an ambiguous diff is left to the node monitor, which matches
// NSpid + the pod's cgroup (vgpu/monitor/pids.py).  flock is released by the kernel when its holder
// dies, so the reference's "unified_lock expired, removing" path is not needed.
//
// The resolved pid is what the share board (board.cpp) records per slot and
// what the node monitor's host-side work needs in a pod: purging dead slots,
// suspend/resume signals and process metrics.  (The temporal limiter charges
// the GPU time of its own marker intervals and needs no pid, limiter.cpp.)
#include <dirent.h>
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <stdarg.h>
#include <sys/file.h>
#include <sys/stat.h>

#include <algorithm>
#include <atomic>
#include <vector>

#include "common.h"
#include "real.h"
#include "state.h"

namespace vgpu {

typedef int (*open_fn)(const char*, int, ...);

namespace {

std::atomic<int> g_phase{0};        // 0 = kfd not opened yet, 1 = bracketing, 2 = done
std::atomic<int> g_host_pid{0};
std::atomic<int> g_host_src{VGPU_HOSTPID_UNVERIFIED};

const char* kfd_dev_path() {
  static const char* p = nullptr;
  const char* v = __atomic_load_n(&p, __ATOMIC_ACQUIRE);
  if (v) return v;
  v = getenv("VGPU_KFD_DEV");
  if (!v || !*v) v = "/dev/kfd";
  __atomic_store_n(&p, v, __ATOMIC_RELEASE);
  return v;
}

open_fn real_open_impl(const char* name) {
  return (open_fn)real_dlsym(RTLD_NEXT, name);
}

open_fn real_open() {
  static open_fn f = nullptr;
  open_fn v = __atomic_load_n(&f, __ATOMIC_ACQUIRE);
  if (!v) {
    v = real_open_impl("open");
    __atomic_store_n(&f, v, __ATOMIC_RELEASE);
  }
  return v;
}

open_fn real_open64() {
  static open_fn f = nullptr;
  open_fn v = __atomic_load_n(&f, __ATOMIC_ACQUIRE);
  if (!v) {
    v = real_open_impl("open64");
    if (!v) v = real_open();
    __atomic_store_n(&f, v, __ATOMIC_RELEASE);
  }
  return v;
}

void list_kfd(std::vector<int>& out) {
  out.clear();
  DIR* d = opendir(kfd_proc_dir());
  if (!d) return;
  while (struct dirent* e = readdir(d)) {
    char* end = nullptr;
    long v = strtol(e->d_name, &end, 10);
    if (end && *end == '\0' && v > 0) out.push_back((int)v);
  }
  closedir(d);
  std::sort(out.begin(), out.end());
}

// Node-wide unified lock (flock on <VGPU_LOCK_DIR|/tmp/vgpulock>/lock).
// Returns the fd to release, or -1 when the directory is absent (no device
// plugin mount: not in a vGPU pod) or the lock could not be taken in 10 s.
int unified_lock() {
  const char* dir = env_first("VGPU_LOCK_DIR");
  if (!dir || !*dir) dir = "/tmp/vgpulock";
  struct stat stt;
  if (stat(dir, &stt) != 0 || !S_ISDIR(stt.st_mode)) return -1;
  char path[512];
  snprintf(path, sizeof path, "%s/lock", dir);
  int fd = real_open()(path, O_RDWR | O_CREAT | O_CLOEXEC, 0666);
  if (fd < 0) return -1;
  const uint64_t t0 = mono_ns();
  while (flock(fd, LOCK_EX | LOCK_NB) != 0) {
    if (errno != EWOULDBLOCK && errno != EINTR) break;
    if (mono_ns() - t0 > 10000000000ull) {
      VLOG_WARN("unified lock %s busy for 10 s; resolving the host pid without it", path);
      close(fd);
      return -1;
    }
    sleep_ns(1000000);
  }
  return fd;
}

void unified_unlock(int fd) {
  if (fd < 0) return;
  flock(fd, LOCK_UN);
  close(fd);
}

int bracketed_kfd_open(open_fn real, const char* path, int flags, mode_t mode) {
  int expected = 0;
  if (!g_phase.compare_exchange_strong(expected, 1)) return real(path, flags, mode);
  const int lk = unified_lock();
  std::vector<int> before, after;
  list_kfd(before);
  const int fd = real(path, flags, mode);
  const int saved_errno = errno;
  list_kfd(after);
  unified_unlock(lk);
  if (fd < 0) {
    g_phase.store(0);  // let a later open try again
    errno = saved_errno;
    return fd;
  }
  std::vector<int> fresh;
  std::set_difference(after.begin(), after.end(), before.begin(), before.end(),
                      std::back_inserter(fresh));
  const int me = getpid();
  int host = 0, src = VGPU_HOSTPID_UNVERIFIED;
  if (fresh.size() == 1) {
    host = fresh[0];
    src = host == me && pid_ns_is_host() ? VGPU_HOSTPID_HOST_NS : VGPU_HOSTPID_KFD_DIFF;
  } else if (std::find(fresh.begin(), fresh.end(), me) != fresh.end() && pid_ns_is_host()) {
    host = me;
    src = VGPU_HOSTPID_HOST_NS;
  } else {
    VLOG_WARN("host pid unresolved: %zu new KFD process entries around our /dev/kfd open%s",
              fresh.size(), lk < 0 ? " (no unified lock)" : "");
  }
  if (host > 0) {
    g_host_pid.store(host);
    g_host_src.store(src);
    VLOG_INFO("host pid %d (container pid %d, %s)", host, me,
              src == VGPU_HOSTPID_KFD_DIFF ? "KFD diff" : "host pid namespace");
    hostpid_publish();
  }
  g_phase.store(2);
  errno = saved_errno;
  return fd;
}

int do_open(open_fn real, const char* path, int flags, mode_t mode) {
  if (__builtin_expect(g_phase.load(std::memory_order_relaxed) != 0 || !path, 1))
    return real(path, flags, mode);
  if (strcmp(path, kfd_dev_path()) != 0) return real(path, flags, mode);
  return bracketed_kfd_open(real, path, flags, mode);
}

}  // namespace

const char* kfd_proc_dir() {
  const char* v = getenv("VGPU_KFD_PROC_DIR");
  return v && *v ? v : "/sys/class/kfd/kfd/proc";
}

// True when this process shares the host's PID namespace.  A pod's namespace
// has no way to see its parent, so the test is indirect: in the initial
// namespace pid 2 is kthreadd (a kernel thread with no command line).
bool pid_ns_is_host() {
  static int cached = -1;
  int c = __atomic_load_n(&cached, __ATOMIC_RELAXED);
  if (c >= 0) return c == 1;
  c = 0;
  if (FILE* f = fopen("/proc/2/status", "r")) {
    char line[128];
    if (fgets(line, sizeof line, f) && strstr(line, "kthreadd")) c = 1;
    fclose(f);
  }
  __atomic_store_n(&cached, c, __ATOMIC_RELAXED);
  return c == 1;
}

int hostpid_resolved(int* src) {
  const int h = g_host_pid.load();
  if (src) *src = h > 0 ? g_host_src.load() : VGPU_HOSTPID_UNVERIFIED;
  return h;
}

int self_host_pid(int* src) {
  int h = hostpid_resolved(src);
  if (h > 0) return h;
  const bool host_ns = pid_ns_is_host();
  if (src) *src = host_ns ? VGPU_HOSTPID_HOST_NS : VGPU_HOSTPID_UNVERIFIED;
  return host_ns ? getpid() : host_pid_of_self();
}

void hostpid_publish() {
  vgpu_proc_slot_t* sl = my_slot();
  if (!sl) return;
  int src = 0;
  const int h = self_host_pid(&src);
  // Never downgrade a pid the node monitor already verified.
  if (src == VGPU_HOSTPID_UNVERIFIED &&
      __atomic_load_n(&sl->host_pid_src, __ATOMIC_ACQUIRE) != VGPU_HOSTPID_UNVERIFIED)
    return;
  __atomic_store_n(&sl->host_pid, h, __ATOMIC_RELAXED);
  __atomic_store_n(&sl->host_pid_src, src, __ATOMIC_RELEASE);
}

std::vector<int> container_host_pids() {
  std::vector<int> out;
  State& s = st();
  if (!s.region) return out;
  for (int i = 0; i < VGPU_MAX_PROCS; ++i) {
    const vgpu_proc_slot_t& sl = s.region->procs[i];
    if (__atomic_load_n(&sl.status, __ATOMIC_ACQUIRE) == VGPU_PROC_FREE) continue;
    if (__atomic_load_n(&sl.host_pid_src, __ATOMIC_ACQUIRE) == VGPU_HOSTPID_UNVERIFIED) continue;
    out.push_back(sl.host_pid);
  }
  return out;
}

void hostpid_after_fork() {
  g_phase.store(0);
  g_host_pid.store(0);
  g_host_src.store(VGPU_HOSTPID_UNVERIFIED);
}

}  // namespace vgpu

using namespace vgpu;

extern "C" {

// Sanitizer runtimes intercept open themselves (host-side race / address
// checking builds, tests/test_shim_robustness.py): those builds leave it alone.
#if !defined(__SANITIZE_THREAD__) && !defined(__SANITIZE_ADDRESS__) && !defined(VGPU_NO_OPEN_HOOK)
__attribute__((visibility("default"))) int open(const char* path, int flags, ...) {
  mode_t mode = 0;
  if (flags & (O_CREAT | O_TMPFILE)) {
    va_list ap;
    va_start(ap, flags);
    mode = (mode_t)va_arg(ap, int);
    va_end(ap);
  }
  return do_open(real_open(), path, flags, mode);
}

__attribute__((visibility("default"))) int open64(const char* path, int flags, ...) {
  mode_t mode = 0;
  if (flags & (O_CREAT | O_TMPFILE)) {
    va_list ap;
    va_start(ap, flags);
    mode = (mode_t)va_arg(ap, int);
    va_end(ap);
  }
  return do_open(real_open64(), path, flags, mode);
}
#endif

// Resolved host pid of this process (0 = unknown) and how it was obtained.
__attribute__((visibility("default"))) int vgpu_self_host_pid(int* src) { return hostpid_resolved(src); }

}  // extern "C"
