#include "region.h"

#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <stddef.h>
#include <sys/file.h>
#include <sys/mman.h>
#include <sys/stat.h>

#include "common.h"

namespace vgpu {

static_assert(sizeof(pthread_mutex_t) <= 64, "mutex must fit its 64-byte slot");
static_assert(sizeof(vgpu_dev_usage_t) == 64, "dev usage is 8 x u64");
static_assert(offsetof(vgpu_shared_region_t, lock) % 8 == 0, "lock alignment");
static_assert(offsetof(vgpu_shared_region_t, procs) % 8 == 0, "procs alignment");

DeviceLimits limits_from_env() {
  DeviceLimits L;
  // Global default limit (applies to every device without an explicit one).
  uint64_t dflt_mem = parse_mem(env_first("VGPU_DEVICE_MEMORY_LIMIT", "CUDA_DEVICE_MEMORY_LIMIT"));
  const char* dflt_cu_s = env_first("VGPU_DEVICE_CU_LIMIT", "CUDA_DEVICE_SM_LIMIT");
  uint32_t dflt_cu = dflt_cu_s ? (uint32_t)atoi(dflt_cu_s) : 0;
  int maxdev = -1;
  for (int i = 0; i < VGPU_MAX_DEVICES; ++i) {
    char a[64], b[64];
    snprintf(a, sizeof a, "VGPU_DEVICE_MEMORY_LIMIT_%d", i);
    snprintf(b, sizeof b, "CUDA_DEVICE_MEMORY_LIMIT_%d", i);
    const char* v = env_first(a, b);
    L.mem_limit[i] = v ? parse_mem(v) : dflt_mem;
    if (v) maxdev = i;
    snprintf(a, sizeof a, "VGPU_DEVICE_MEMORY_PHYSICAL_%d", i);
    v = env_first(a);
    L.mem_physical[i] = v ? parse_mem(v) : 0;
    snprintf(a, sizeof a, "VGPU_DEVICE_CU_LIMIT_%d", i);
    v = env_first(a);
    L.cu_limit[i] = v ? (uint32_t)atoi(v) : dflt_cu;
    if (v) maxdev = i > maxdev ? i : maxdev;
    snprintf(a, sizeof a, "VGPU_CU_MASK_%d", i);
    v = env_first(a);
    if (v) {
      if (parse_cu_mask(v, L.cu_mask[i], VGPU_CU_MASK_WORDS) < 0) {
        VLOG_WARN("ignoring malformed %s=%s", a, v);
        memset(L.cu_mask[i], 0, sizeof(L.cu_mask[i]));
      }
      maxdev = i > maxdev ? i : maxdev;
    }
    snprintf(a, sizeof a, "VGPU_DEVICE_UUID_%d", i);
    v = env_first(a);
    if (v) snprintf(L.uuid[i], VGPU_UUID_LEN, "%s", v);
  }
  L.num_devices = maxdev + 1;
  if (L.num_devices == 0 && (dflt_mem || dflt_cu)) L.num_devices = VGPU_MAX_DEVICES;
  L.oversubscribe = env_bool(env_first("VGPU_OVERSUBSCRIBE", "CUDA_OVERSUBSCRIBE"), false);
  L.suspend_evict = env_bool(env_first("VGPU_SUSPEND_EVICT"), false);
  const char* p = env_first("VGPU_TASK_PRIORITY", "CUDA_TASK_PRIORITY");
  L.priority = p ? atoi(p) : 1;
  const char* pol = env_first("GPU_CORE_UTILIZATION_POLICY");
  L.core_policy = 0;
  if (pol && !strcasecmp(pol, "force")) L.core_policy = 1;
  if (pol && !strcasecmp(pol, "disable")) L.core_policy = 2;
  return L;
}

static void init_mutex(vgpu_shared_region_t* r) {
  pthread_mutexattr_t a;
  pthread_mutexattr_init(&a);
  pthread_mutexattr_setpshared(&a, PTHREAD_PROCESS_SHARED);
  pthread_mutexattr_setrobust(&a, PTHREAD_MUTEX_ROBUST);
  pthread_mutex_init(&r->lock.m, &a);
  pthread_mutexattr_destroy(&a);
}

static void write_limits(vgpu_shared_region_t* r, const DeviceLimits& L) {
  r->num_devices = L.num_devices;
  r->oversubscribe = L.oversubscribe;
  r->priority = L.priority;
  r->core_policy = L.core_policy;
  for (int i = 0; i < VGPU_MAX_DEVICES; ++i) {
    vgpu_device_cfg_t& d = r->dev[i];
    d.mem_limit = L.mem_limit[i];
    d.mem_physical = L.mem_physical[i];
    d.flags = L.suspend_evict ? (d.flags | VGPU_DEV_FLAG_SUSPEND_EVICT) : (d.flags & ~VGPU_DEV_FLAG_SUSPEND_EVICT);
    d.cu_limit = L.cu_limit[i];
    memcpy(d.cu_mask, L.cu_mask[i], sizeof(d.cu_mask));
    if (L.uuid[i][0]) memcpy(d.uuid, L.uuid[i], VGPU_UUID_LEN);
  }
}

static bool limits_differ(const vgpu_shared_region_t* r, const DeviceLimits& L) {
  for (int i = 0; i < VGPU_MAX_DEVICES; ++i) {
    if (r->dev[i].mem_limit != L.mem_limit[i]) return true;
    if (r->dev[i].mem_physical != L.mem_physical[i]) return true;
    if (r->dev[i].cu_limit != L.cu_limit[i]) return true;
    if (memcmp(r->dev[i].cu_mask, L.cu_mask[i], sizeof(L.cu_mask[i]))) return true;
  }
  return false;
}

static void init_region(vgpu_shared_region_t* r, const DeviceLimits* lim) {
  memset(r, 0, sizeof(*r));
  r->magic = VGPU_REGION_MAGIC;
  r->version = VGPU_REGION_VERSION;
  r->struct_size = (uint32_t)sizeof(*r);
  init_mutex(r);
  r->create_ns = real_ns();
  r->recent_kernel = 0;
  r->utilization_switch = 1;  // throttle until the monitor says otherwise
  if (lim) write_limits(r, *lim);
  __atomic_store_n(&r->initialized, 1, __ATOMIC_RELEASE);
}

vgpu_shared_region_t* region_map(const char* path, const DeviceLimits* lim, int* fd_out) {
  const size_t sz = sizeof(vgpu_shared_region_t);
  *fd_out = -1;
  if (!path || !*path) {
    void* p = mmap(nullptr, sz, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) return nullptr;
    auto* r = (vgpu_shared_region_t*)p;
    init_region(r, lim);
    return r;
  }
  int fd = open(path, lim ? (O_RDWR | O_CREAT) : O_RDWR, 0666);
  if (fd < 0) {
    VLOG_WARN("cannot open shared region %s: %s", path, strerror(errno));
    return nullptr;
  }
  // Serialise creation/initialisation across processes with an advisory lock.
  if (flock(fd, LOCK_EX) != 0) VLOG_WARN("flock(%s) failed: %s", path, strerror(errno));
  struct stat st;
  fstat(fd, &st);
  bool fresh = (size_t)st.st_size < sz;
  if (fresh) {
    if (!lim) {
      flock(fd, LOCK_UN);
      close(fd);
      return nullptr;  // attach-only on a file that was never initialised
    }
    if (ftruncate(fd, (off_t)sz) != 0) {
      VLOG_ERR("ftruncate(%s) failed: %s", path, strerror(errno));
      flock(fd, LOCK_UN);
      close(fd);
      return nullptr;
    }
  }
  void* p = mmap(nullptr, sz, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) {
    VLOG_ERR("mmap(%s) failed: %s", path, strerror(errno));
    flock(fd, LOCK_UN);
    close(fd);
    return nullptr;
  }
  auto* r = (vgpu_shared_region_t*)p;
  bool bad = r->magic != VGPU_REGION_MAGIC || r->version != VGPU_REGION_VERSION ||
             r->struct_size != sz || !r->initialized;
  if (lim) {
    if (fresh || bad) {
      if (bad && !fresh) VLOG_WARN("shared region %s has a stale layout; reinitialising", path);
      init_region(r, lim);
    } else if (limits_differ(r, *lim)) {
      VLOG_WARN("Limit inconsistency between %s and the environment; environment wins", path);
      write_limits(r, *lim);
    }
  } else if (bad) {
    munmap(p, sz);
    flock(fd, LOCK_UN);
    close(fd);
    return nullptr;
  }
  flock(fd, LOCK_UN);
  *fd_out = fd;
  return r;
}

void region_unmap(vgpu_shared_region_t* r, int fd) {
  if (r) munmap(r, sizeof(*r));
  if (fd >= 0) close(fd);
}

static bool pid_alive(int pid) {
  if (pid <= 0) return false;
  if (kill(pid, 0) == 0) return true;
  return errno == EPERM;  // exists but not ours
}

int region_purge_dead_locked(vgpu_shared_region_t* r, bool host_ns) {
  int purged = 0, live = 0;
  for (int i = 0; i < VGPU_MAX_PROCS; ++i) {
    vgpu_proc_slot_t& s = r->procs[i];
    if (s.status == VGPU_PROC_FREE) continue;
    // A host-side caller cannot judge a slot whose host pid was never
    // verified (it is a container pid, meaningless in the host namespace).
    if (host_ns && s.host_pid_src == VGPU_HOSTPID_UNVERIFIED) { ++live; continue; }
    int pid = host_ns ? s.host_pid : s.pid;
    if (!pid_alive(pid)) {
      VLOG_INFO("purging slot %d of exited pid %d", i, pid);
      memset(&s, 0, sizeof(s));
      ++purged;
    } else {
      ++live;
    }
  }
  r->proc_num = live;
  return purged;
}

int region_lock(vgpu_shared_region_t* r) {
  int rc = pthread_mutex_lock(&r->lock.m);
  if (rc == EOWNERDEAD) {
    VLOG_WARN("shared region lock owner died; recovering");
    pthread_mutex_consistent(&r->lock.m);
    region_purge_dead_locked(r, false);
    rc = 0;
  }
  return rc;
}

void region_unlock(vgpu_shared_region_t* r) { pthread_mutex_unlock(&r->lock.m); }

int region_claim_slot(vgpu_shared_region_t* r, int pid, int host_pid, int priority) {
  if (region_lock(r) != 0) return -1;
  int found = -1, free_slot = -1;
  for (int i = 0; i < VGPU_MAX_PROCS; ++i) {
    if (r->procs[i].status != VGPU_PROC_FREE && r->procs[i].pid == pid) { found = i; break; }
    if (free_slot < 0 && r->procs[i].status == VGPU_PROC_FREE) free_slot = i;
  }
  if (found < 0 && free_slot < 0) {
    region_purge_dead_locked(r, false);
    for (int i = 0; i < VGPU_MAX_PROCS; ++i)
      if (r->procs[i].status == VGPU_PROC_FREE) { free_slot = i; break; }
  }
  int slot = found >= 0 ? found : free_slot;
  if (slot >= 0) {
    vgpu_proc_slot_t& s = r->procs[slot];
    if (found < 0) memset(&s, 0, sizeof(s));  // stale pid reuse: fresh counters
    s.pid = pid;
    s.host_pid = host_pid;
    s.host_pid_src = VGPU_HOSTPID_UNVERIFIED;
    s.priority = priority;
    s.start_ns = mono_ns();
    __atomic_store_n(&s.status, VGPU_PROC_RUNNING, __ATOMIC_RELEASE);
    int live = 0;
    for (int i = 0; i < VGPU_MAX_PROCS; ++i) live += r->procs[i].status != VGPU_PROC_FREE;
    r->proc_num = live;
  }
  region_unlock(r);
  return slot;
}

void region_release_slot(vgpu_shared_region_t* r, int slot) {
  if (slot < 0 || slot >= VGPU_MAX_PROCS) return;
  if (region_lock(r) != 0) return;
  memset(&r->procs[slot], 0, sizeof(r->procs[slot]));
  int live = 0;
  for (int i = 0; i < VGPU_MAX_PROCS; ++i) live += r->procs[i].status != VGPU_PROC_FREE;
  r->proc_num = live;
  region_unlock(r);
}

int region_purge_dead(vgpu_shared_region_t* r, bool host_ns) {
  if (region_lock(r) != 0) return -1;
  int n = region_purge_dead_locked(r, host_ns);
  region_unlock(r);
  return n;
}

uint64_t region_device_used(const vgpu_shared_region_t* r, int dev) {
  uint64_t sum = 0;
  for (int i = 0; i < VGPU_MAX_PROCS; ++i) {
    if (r->procs[i].status == VGPU_PROC_FREE) continue;
    sum += __atomic_load_n(&r->procs[i].used[dev].total_bytes, __ATOMIC_RELAXED);
  }
  return sum;
}

uint64_t region_device_host_used(const vgpu_shared_region_t* r, int dev) {
  uint64_t sum = 0;
  for (int i = 0; i < VGPU_MAX_PROCS; ++i) {
    if (r->procs[i].status == VGPU_PROC_FREE) continue;
    sum += __atomic_load_n(&r->procs[i].used[dev].host_bytes, __ATOMIC_RELAXED);
  }
  return sum;
}

int host_pid_of_self() {
  FILE* f = fopen("/proc/self/status", "r");
  if (!f) return getpid();
  char line[256];
  int pid = getpid();
  while (fgets(line, sizeof line, f)) {
    if (!strncmp(line, "NSpid:", 6)) {
      int v = 0;
      if (sscanf(line + 6, "%d", &v) == 1 && v > 0) pid = v;
      break;
    }
  }
  fclose(f);
  return pid;
}

void region_fill_layout(vgpu_region_layout_t* o) {
  o->region_size = sizeof(vgpu_shared_region_t);
  o->proc_slot_size = sizeof(vgpu_proc_slot_t);
  o->dev_usage_size = sizeof(vgpu_dev_usage_t);
  o->device_cfg_size = sizeof(vgpu_device_cfg_t);
  o->off_lock = offsetof(vgpu_shared_region_t, lock);
  o->off_num_devices = offsetof(vgpu_shared_region_t, num_devices);
  o->off_recent_kernel = offsetof(vgpu_shared_region_t, recent_kernel);
  o->off_dev = offsetof(vgpu_shared_region_t, dev);
  o->off_procs = offsetof(vgpu_shared_region_t, procs);
  o->mutex_size = sizeof(pthread_mutex_t);
}

}  // namespace vgpu
