// JSON/env-driven fake of the ROCr (HSA) runtime, for CPU-only tests of the
// enforcement library.  Mirrors the role of the reference's fake libcndev.so
// (pkg/device-plugin/mlu/cndev/mock/cndev.c:22-39): a real shared object with
// the vendor ABI, answering from a fixture instead of hardware.
//
// Built as libhsa-runtime64.so.1 (SONAME) with the ROCR_1 symbol version.
// Fixture: VGPU_FAKE_GPUS (default 1), VGPU_FAKE_CUS (256), VGPU_FAKE_XCC (8).
//
// Like ROCr, every exported queue / pool entry point dispatches through an
// HsaApiTable, and hsa_init() hands that table to the OnLoad() of every
// library named in HSA_TOOLS_LIB — the tools-library interception path of
// the enforcement library (native/shim/hooks_hsa.cpp).
#include <dlfcn.h>
#include <fcntl.h>
#include <stdarg.h>
#include <stdio.h>
#include <sys/stat.h>
#include <unistd.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#define AMD_INTERNAL_BUILD 1
#include <hsa/hsa_api_trace.h>
#undef AMD_INTERNAL_BUILD
#include <stdlib.h>
#include <string.h>

#include <map>
#include <string>

#include <atomic>
#include <mutex>
#include <vector>

namespace {

struct FakeQueue {
  hsa_queue_t q;
  uint64_t agent;
  uint32_t mask[8];
  uint32_t mask_bits;
  int alive;
  int intercept;  // created by hsa_amd_queue_intercept_create
  hsa_amd_queue_intercept_handler handler;
  void* hdata;
};

// Intercept queues (ROCr's InterceptQueue, reached only through the AMD
// extension table): a submission (fake_hsa_submit, standing in for the
// doorbell write) hands the packets to the registered handler, which writes
// what it lets through to the "hardware" -- here a counter of kernel-dispatch
// packets.
std::atomic<uint64_t> g_dispatched{0};
void fake_writer(const void* pkts, uint64_t n) {
  const auto* p = static_cast<const hsa_kernel_dispatch_packet_t*>(pkts);
  for (uint64_t i = 0; i < n; ++i)
    if ((p[i].header & 0xff) == HSA_PACKET_TYPE_KERNEL_DISPATCH) g_dispatched.fetch_add(1);
}

std::mutex g_mu;
std::vector<FakeQueue*> g_queues;

int env_int(const char* n, int d) {
  const char* v = getenv(n);
  return v && *v ? atoi(v) : d;
}

// Pools: CPU agent (handle 1) owns pool 2; GPU agent 100+i owns pool 200+i.
std::map<uintptr_t, std::pair<uint64_t, uint64_t>> g_pool_allocs;  // ptr -> (pool, size)
std::map<uint64_t, uint64_t> g_pool_used;
uintptr_t g_pool_next = 0x600000000000ull;

hsa_status_t impl_queue_create(hsa_agent_t agent, uint32_t size, hsa_queue_type32_t type,
                               void (*callback)(hsa_status_t, hsa_queue_t*, void*), void* data,
                               uint32_t priv, uint32_t group, hsa_queue_t** queue);
hsa_status_t impl_queue_destroy(hsa_queue_t* q);
hsa_status_t impl_cu_set_mask(const hsa_queue_t* q, uint32_t bits, const uint32_t* mask);
hsa_status_t impl_pool_allocate(hsa_amd_memory_pool_t pool, size_t size, uint32_t flags, void** ptr);
hsa_status_t impl_pool_free(void* ptr);
hsa_status_t impl_intercept_create(hsa_agent_t agent, uint32_t size, hsa_queue_type32_t type,
                                   void (*callback)(hsa_status_t, hsa_queue_t*, void*), void* data,
                                   uint32_t priv, uint32_t group, hsa_queue_t** queue);
hsa_status_t impl_intercept_register(hsa_queue_t* q, hsa_amd_queue_intercept_handler h, void* data);

CoreApiTable g_core;
AmdExtTable g_ext;
HsaApiTable g_api;
std::once_flag g_table_once;
int g_tools_loaded = 0;

void setup_table() {
  std::call_once(g_table_once, [] {
    memset(&g_core, 0, sizeof g_core);
    memset(&g_ext, 0, sizeof g_ext);
    memset(&g_api, 0, sizeof g_api);
    g_core.hsa_queue_create_fn = impl_queue_create;
    g_core.hsa_queue_destroy_fn = impl_queue_destroy;
    g_ext.hsa_amd_queue_cu_set_mask_fn = impl_cu_set_mask;
    g_ext.hsa_amd_memory_pool_allocate_fn = impl_pool_allocate;
    g_ext.hsa_amd_memory_pool_free_fn = impl_pool_free;
    g_ext.hsa_amd_queue_intercept_create_fn = impl_intercept_create;
    g_ext.hsa_amd_queue_intercept_register_fn = impl_intercept_register;
    g_api.core_ = &g_core;
    g_api.amd_ext_ = &g_ext;
    const char* tools = getenv("HSA_TOOLS_LIB");
    if (!tools || !*tools) return;
    std::string all(tools);
    size_t pos = 0;
    while (pos <= all.size()) {
      size_t end = all.find_first_of(" :", pos);
      if (end == std::string::npos) end = all.size();
      std::string lib = all.substr(pos, end - pos);
      pos = end + 1;
      if (lib.empty()) continue;
      void* h = dlopen(lib.c_str(), RTLD_NOW);
      if (!h) continue;
      typedef bool (*onload_t)(void*, uint64_t, uint64_t, const char* const*);
      auto fn = (onload_t)dlsym(h, "OnLoad");
      if (fn && fn(&g_api, 1, 0, nullptr)) ++g_tools_loaded;
    }
  });
}

// Fake KFD driver: opening VGPU_FAKE_KFD_DEV creates this process's entry in
// the KFD proc directory (VGPU_KFD_PROC_DIR) named by VGPU_FAKE_HOST_PID, the
// way amdgpu's kfd_open() creates /sys/class/kfd/kfd/proc/<host pid> inside
// the open() call.  VGPU_FAKE_KFD_NOISE=<pid> adds an unrelated process's
// entry in the same instant (an ambiguous diff).
int fake_kfd_open(const char* path, int flags, mode_t mode) {
  typedef int (*open_t)(const char*, int, ...);
  static open_t real = (open_t)dlsym(RTLD_NEXT, "open");
  const char* dev = getenv("VGPU_FAKE_KFD_DEV");
  if (dev && *dev && path && !strcmp(path, dev)) {
    const char* dir = getenv("VGPU_KFD_PROC_DIR");
    const char* hp = getenv("VGPU_FAKE_HOST_PID");
    char p[512];
    if (dir && hp) {
      snprintf(p, sizeof p, "%s/%s", dir, hp);
      mkdir(p, 0755);
    }
    const char* noise = getenv("VGPU_FAKE_KFD_NOISE");
    if (dir && noise && *noise) {
      snprintf(p, sizeof p, "%s/%s", dir, noise);
      mkdir(p, 0755);
    }
  }
  return real(path, flags, mode);
}

}  // namespace

extern "C" {

int open(const char* path, int flags, ...) {
  mode_t mode = 0;
  if (flags & O_CREAT) {
    va_list ap;
    va_start(ap, flags);
    mode = (mode_t)va_arg(ap, int);
    va_end(ap);
  }
  return fake_kfd_open(path, flags, mode);
}

hsa_status_t hsa_init() {
  setup_table();
  // ROCr opens the KFD character device first thing in hsa_init.
  const char* dev = getenv("VGPU_FAKE_KFD_DEV");
  static int kfd_fd = -1;
  if (dev && *dev && kfd_fd < 0) kfd_fd = open(dev, O_RDWR | O_CLOEXEC);
  return HSA_STATUS_SUCCESS;
}
hsa_status_t hsa_shut_down() { return HSA_STATUS_SUCCESS; }

hsa_status_t hsa_iterate_agents(hsa_status_t (*cb)(hsa_agent_t, void*), void* data) {
  // One CPU agent first (handle 1), then the GPUs (handles 100+i), as ROCr does.
  hsa_agent_t cpu{1};
  hsa_status_t rc = cb(cpu, data);
  if (rc != HSA_STATUS_SUCCESS) return rc;
  int n = env_int("VGPU_FAKE_GPUS", 1);
  for (int i = 0; i < n; ++i) {
    hsa_agent_t a{(uint64_t)(100 + i)};
    rc = cb(a, data);
    if (rc != HSA_STATUS_SUCCESS) return rc;
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t hsa_agent_get_info(hsa_agent_t agent, hsa_agent_info_t attr, void* value) {
  bool gpu = agent.handle >= 100;
  switch ((int)attr) {
    case HSA_AGENT_INFO_DEVICE:
      *(hsa_device_type_t*)value = gpu ? HSA_DEVICE_TYPE_GPU : HSA_DEVICE_TYPE_CPU;
      return HSA_STATUS_SUCCESS;
    case HSA_AMD_AGENT_INFO_COMPUTE_UNIT_COUNT:
      *(uint32_t*)value = gpu ? (uint32_t)env_int("VGPU_FAKE_CUS", 256) : 8;
      return HSA_STATUS_SUCCESS;
    case HSA_AMD_AGENT_INFO_NUM_XCC:
      *(uint32_t*)value = gpu ? (uint32_t)env_int("VGPU_FAKE_XCC", 8) : 1;
      return HSA_STATUS_SUCCESS;
    case HSA_AMD_AGENT_INFO_DRIVER_UID:
      *(uint32_t*)value = gpu ? (uint32_t)(1000 + agent.handle - 100) : 0;
      return HSA_STATUS_SUCCESS;
    default:
      return HSA_STATUS_ERROR_INVALID_ARGUMENT;
  }
}

hsa_status_t hsa_amd_agent_iterate_memory_pools(hsa_agent_t agent,
                                                hsa_status_t (*cb)(hsa_amd_memory_pool_t, void*),
                                                void* data) {
  hsa_amd_memory_pool_t p{agent.handle >= 100 ? 200 + (agent.handle - 100) : 2};
  return cb(p, data);
}

hsa_status_t hsa_amd_memory_pool_get_info(hsa_amd_memory_pool_t pool,
                                          hsa_amd_memory_pool_info_t attr, void* value) {
  if (attr == HSA_AMD_MEMORY_POOL_INFO_SEGMENT) {
    *(hsa_amd_segment_t*)value = HSA_AMD_SEGMENT_GLOBAL;
    return HSA_STATUS_SUCCESS;
  }
  return HSA_STATUS_ERROR_INVALID_ARGUMENT;
}

// Exported entry points dispatch through the API table, as ROCr's do.
hsa_status_t hsa_queue_create(hsa_agent_t agent, uint32_t size, hsa_queue_type32_t type,
                              void (*callback)(hsa_status_t, hsa_queue_t*, void*), void* data,
                              uint32_t priv, uint32_t group, hsa_queue_t** queue) {
  setup_table();
  return g_core.hsa_queue_create_fn(agent, size, type, callback, data, priv, group, queue);
}
hsa_status_t hsa_queue_destroy(hsa_queue_t* q) {
  setup_table();
  return g_core.hsa_queue_destroy_fn(q);
}
hsa_status_t hsa_amd_queue_cu_set_mask(const hsa_queue_t* q, uint32_t bits, const uint32_t* mask) {
  setup_table();
  return g_ext.hsa_amd_queue_cu_set_mask_fn(q, bits, mask);
}
hsa_status_t hsa_amd_memory_pool_allocate(hsa_amd_memory_pool_t pool, size_t size, uint32_t flags,
                                          void** ptr) {
  setup_table();
  return g_ext.hsa_amd_memory_pool_allocate_fn(pool, size, flags, ptr);
}
hsa_status_t hsa_amd_memory_pool_free(void* ptr) {
  setup_table();
  return g_ext.hsa_amd_memory_pool_free_fn(ptr);
}

// Signals: a heap word; every fake asynchronous operation completes before it returns.
hsa_status_t hsa_signal_create(hsa_signal_value_t initial, uint32_t, const hsa_agent_t*, hsa_signal_t* sig) {
  sig->handle = (uint64_t)(uintptr_t)new int64_t(initial);
  return HSA_STATUS_SUCCESS;
}
hsa_status_t hsa_signal_destroy(hsa_signal_t sig) {
  delete (int64_t*)(uintptr_t)sig.handle;
  return HSA_STATUS_SUCCESS;
}
hsa_signal_value_t hsa_signal_wait_scacquire(hsa_signal_t sig, hsa_signal_condition_t, hsa_signal_value_t,
                                             uint64_t, hsa_wait_state_t) {
  return *(int64_t*)(uintptr_t)sig.handle;
}
// KFD SVM: attributes are accepted; a prefetch moves the fake HIP's managed
// range bookkeeping (VRAM use) at VGPU_FAKE_SVM_GBPS (default: instantly).
hsa_status_t hsa_amd_svm_attributes_set(void*, size_t, hsa_amd_svm_attribute_pair_t*, size_t) {
  return HSA_STATUS_SUCCESS;
}
hsa_status_t hsa_amd_svm_prefetch_async(void* ptr, size_t size, hsa_agent_t agent, uint32_t, const hsa_signal_t*,
                                        hsa_signal_t done) {
  typedef int (*move_t)(const void*, uint64_t, int);
  static move_t move = (move_t)dlsym(RTLD_DEFAULT, "fake_hip_svm_move");
  if (!move || move(ptr, size, agent.handle >= 100 ? 1 : 0) < 0) return HSA_STATUS_ERROR_INVALID_ARGUMENT;
  if (int gbps = env_int("VGPU_FAKE_SVM_GBPS", 0)) usleep((useconds_t)(size / (gbps * 1000.0)));
  if (done.handle) --*(int64_t*)(uintptr_t)done.handle;
  return HSA_STATUS_SUCCESS;
}

// ---- test introspection ----
uint64_t fake_hsa_pool_used(int dev) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_pool_used.find(200 + (uint64_t)dev);
  return it == g_pool_used.end() ? 0 : it->second;
}
int fake_hsa_tools_loaded() { return g_tools_loaded; }

}  // extern "C"

namespace {

hsa_status_t impl_pool_allocate(hsa_amd_memory_pool_t pool, size_t size, uint32_t, void** ptr) {
  if (!ptr || size == 0) return HSA_STATUS_ERROR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> g(g_mu);
  uintptr_t a = g_pool_next;
  g_pool_next += ((size + 4095) / 4096) * 4096 + 4096;
  g_pool_allocs[a] = {pool.handle, size};
  g_pool_used[pool.handle] += size;
  *ptr = (void*)a;
  return HSA_STATUS_SUCCESS;
}

hsa_status_t impl_pool_free(void* ptr) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_pool_allocs.find((uintptr_t)ptr);
  if (it == g_pool_allocs.end()) return HSA_STATUS_ERROR_INVALID_ARGUMENT;
  g_pool_used[it->second.first] -= it->second.second;
  g_pool_allocs.erase(it);
  return HSA_STATUS_SUCCESS;
}

hsa_status_t impl_queue_create(hsa_agent_t agent, uint32_t size, hsa_queue_type32_t type,
                               void (*callback)(hsa_status_t, hsa_queue_t*, void*), void* data,
                               uint32_t priv, uint32_t group, hsa_queue_t** queue) {
  auto* fq = new FakeQueue();
  memset(fq, 0, sizeof(*fq));
  fq->agent = agent.handle;
  fq->q.size = size;
  fq->alive = 1;
  std::lock_guard<std::mutex> g(g_mu);
  g_queues.push_back(fq);
  *queue = &fq->q;
  return HSA_STATUS_SUCCESS;
}

hsa_status_t impl_intercept_create(hsa_agent_t agent, uint32_t size, hsa_queue_type32_t type,
                                   void (*callback)(hsa_status_t, hsa_queue_t*, void*), void* data,
                                   uint32_t priv, uint32_t group, hsa_queue_t** queue) {
  hsa_status_t rc = impl_queue_create(agent, size, type, callback, data, priv, group, queue);
  if (rc == HSA_STATUS_SUCCESS) reinterpret_cast<FakeQueue*>(*queue)->intercept = 1;
  return rc;
}

hsa_status_t impl_intercept_register(hsa_queue_t* q, hsa_amd_queue_intercept_handler h, void* data) {
  std::lock_guard<std::mutex> g(g_mu);
  for (auto* fq : g_queues) {
    if (&fq->q != q) continue;
    if (!fq->intercept) return HSA_STATUS_ERROR_INVALID_QUEUE;
    fq->handler = h;
    fq->hdata = data;
    return HSA_STATUS_SUCCESS;
  }
  return HSA_STATUS_ERROR_INVALID_QUEUE;
}

hsa_status_t impl_queue_destroy(hsa_queue_t* q) {
  std::lock_guard<std::mutex> g(g_mu);
  for (auto* fq : g_queues)
    if (&fq->q == q) fq->alive = 0;
  return HSA_STATUS_SUCCESS;
}

hsa_status_t impl_cu_set_mask(const hsa_queue_t* q, uint32_t bits, const uint32_t* mask) {
  if (bits % 32) return HSA_STATUS_ERROR_INVALID_ARGUMENT;
  if (bits && !mask) return HSA_STATUS_ERROR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> g(g_mu);
  for (auto* fq : g_queues) {
    if (&fq->q != q) continue;
    memset(fq->mask, 0, sizeof(fq->mask));
    fq->mask_bits = bits;
    for (uint32_t w = 0; w < bits / 32 && w < 8; ++w) fq->mask[w] = mask[w];
    return HSA_STATUS_SUCCESS;
  }
  return HSA_STATUS_ERROR_INVALID_QUEUE;
}

}  // namespace

extern "C" {

// The doorbell write of `n` packets on queue `q` (see fake_writer).
void fake_hsa_submit(hsa_queue_t* q, const void* pkts, uint64_t n) {
  hsa_amd_queue_intercept_handler h = nullptr;
  void* data = nullptr;
  {
    std::lock_guard<std::mutex> g(g_mu);
    for (auto* fq : g_queues)
      if (&fq->q == q) {
        h = fq->handler;
        data = fq->hdata;
      }
  }
  if (h) h(pkts, n, 0, data, fake_writer);
  else fake_writer(pkts, n);
}
uint64_t fake_hsa_dispatched() { return g_dispatched.load(); }
int fake_hsa_intercept_queues() {
  std::lock_guard<std::mutex> g(g_mu);
  int n = 0;
  for (auto* fq : g_queues) n += fq->intercept && fq->alive;
  return n;
}

int fake_hsa_queue_count() {
  std::lock_guard<std::mutex> g(g_mu);
  return (int)g_queues.size();
}

// Returns number of 32-bit words written (0 = "all CUs").
int fake_hsa_queue_mask(int idx, uint32_t* out, int max_words, uint64_t* agent) {
  std::lock_guard<std::mutex> g(g_mu);
  if (idx < 0 || idx >= (int)g_queues.size()) return -1;
  FakeQueue* fq = g_queues[idx];
  int n = (int)fq->mask_bits / 32;
  for (int w = 0; w < n && w < max_words; ++w) out[w] = fq->mask[w];
  if (agent) *agent = fq->agent;
  return n;
}

}  // extern "C"
