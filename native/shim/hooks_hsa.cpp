// ROCr (HSA) interposers: catch every hardware queue the process creates so the
// container's CU mask is applied before the first dispatch (and keep the
// application from widening it), and charge device-memory pool allocations
// that bypass the HIP allocation hooks (runtime kernarg / staging buffers,
// direct HSA users) to the container.
//
// The CU-mask half has no reference counterpart (CUDA offers no per-stream SM
// mask); it is the MI355X replacement for the time-sliced SM limiter
// (SURVEY.md §2.6 E1f, §7.2 step 3(a)).  The pool half is the HSA-level
// accounting of SURVEY.md §7.4 item 1 (reference: allocator.c tracks context /
// module / buffer bytes separately, E1d).
//
// Two ways in, one implementation:
//  * LD_PRELOAD / ld.so.preload: the exported hsa_* below interpose on the
//    HIP runtime's PLT calls into libhsa-runtime64.
//  * HSA_TOOLS_LIB=libvgpu.so: ROCr calls OnLoad() with its API table before
//    the first queue exists, and we swap the table entries.  Every caller —
//    including code that resolved hsa_* by hand — dispatches through that
//    table (the rocprofiler mechanism; SURVEY.md §2.6 E1a "HSA tools-lib
//    OnLoad").  Once the table is patched the PLT interposers pass through,
//    so nothing is applied or charged twice.
// The installed header picks its sibling includes by this macro.
#define AMD_INTERNAL_BUILD 1
#include <hsa/hsa_api_trace.h>
#undef AMD_INTERNAL_BUILD

#include <dlfcn.h>
#include <execinfo.h>

#include <atomic>
#include <mutex>
#include <unordered_map>

#include "common.h"
#include "real.h"
#include "state.h"

namespace vgpu {
bool cumask_intersect(const hsa_queue_t* q, uint32_t* bits, const uint32_t* in, uint32_t* out);
int cumask_hip_index_for_pool(uint64_t pool_handle);
int cumask_hip_index_for_agent(uint64_t agent_handle);
std::atomic<uint64_t> g_hsa_dispatches{0};     // kernel dispatches seen by intercept queues
std::atomic<int> g_hsa_intercepted_queues{0};

namespace {

struct HsaTable {
  decltype(&::hsa_queue_create) queue_create = nullptr;
  decltype(&::hsa_queue_destroy) queue_destroy = nullptr;
  decltype(&::hsa_amd_queue_cu_set_mask) cu_set_mask = nullptr;
  decltype(&::hsa_amd_memory_pool_allocate) pool_allocate = nullptr;
  decltype(&::hsa_amd_memory_pool_free) pool_free = nullptr;
  decltype(&::hsa_amd_queue_intercept_create) intercept_create = nullptr;
  decltype(&::hsa_amd_queue_intercept_register) intercept_register = nullptr;
};
HsaTable g_orig;                    // ROCr's entries, saved by OnLoad
std::atomic<bool> g_table_mode{false};

hsa_status_t queue_create_impl(decltype(&::hsa_queue_create) real, hsa_agent_t agent, uint32_t size,
                               hsa_queue_type32_t type,
                               void (*callback)(hsa_status_t, hsa_queue_t*, void*), void* data,
                               uint32_t private_segment_size, uint32_t group_segment_size,
                               hsa_queue_t** queue) {
  ensure_init();
  hsa_status_t rc = real(agent, size, type, callback, data, private_segment_size,
                         group_segment_size, queue);
  if (rc == HSA_STATUS_SUCCESS && queue && *queue) cumask_on_queue_created(&agent, *queue);
  return rc;
}

hsa_status_t cu_set_mask_impl(decltype(&::hsa_amd_queue_cu_set_mask) real, const hsa_queue_t* queue,
                              uint32_t num_cu_mask_count, const uint32_t* cu_mask) {
  ensure_init();
  uint32_t bits = num_cu_mask_count;
  uint32_t merged[VGPU_CU_MASK_WORDS * 2] = {};
  if (num_cu_mask_count <= VGPU_CU_MASK_WORDS * 64 &&
      cumask_intersect(queue, &bits, cu_mask, merged))
    return real(queue, bits, merged);
  return real(queue, num_cu_mask_count, cu_mask);
}

// Who called hsa_amd_memory_pool_allocate.  The HIP runtime and ROCr itself
// (kernarg pools, staging buffers, scratch, code objects) are charged without
// being refused: refusing them would fail a kernel launch or a copy, not an
// allocation the application can handle.  Every other caller — code using
// HSA directly, libraries that bypass hipMalloc — is refused past the cap,
// exactly like hipMalloc.  Decided once per calling object.
bool runtime_caller(const void* ret_addr) {
  if (!ret_addr) return true;  // reached through the API table by hand-resolved code or ROCr
  static std::mutex mu;
  static std::unordered_map<const void*, bool> cache;  // object base -> runtime?
  Dl_info di;
  if (!dladdr(ret_addr, &di) || !di.dli_fbase) return true;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(di.dli_fbase);
  if (it != cache.end()) return it->second;
  const char* f = di.dli_fname ? di.dli_fname : "";
  const bool rt = strstr(f, "libamdhip64") || strstr(f, "libhsa-runtime64") || is_own_address((void*)ret_addr);
  cache.emplace(di.dli_fbase, rt);
  return rt;
}

thread_local const void* tl_pool_caller = nullptr;  // PLT caller, handed to the table entry

hsa_status_t pool_allocate_impl(decltype(&::hsa_amd_memory_pool_allocate) real,
                                hsa_amd_memory_pool_t pool, size_t size, uint32_t flags,
                                void** ptr, const void* caller) {
  // Allocations made inside a HIP allocation hook are already charged there.
  if (tl_in_hip_alloc || size == 0) return real(pool, size, flags, ptr);
  ensure_init();
  if (!st().enabled) return real(pool, size, flags, ptr);
  const int dev = cumask_hip_index_for_pool(pool.handle);
  if (dev < 0) return real(pool, size, flags, ptr);  // host pool or a device outside the container
  if (!runtime_caller(caller)) {
    charge_context(dev);
    if (!mem_reserve(dev, size, kDeviceBuf)) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
    hsa_status_t rc = real(pool, size, flags, ptr);
    if (rc != HSA_STATUS_SUCCESS || !ptr || !*ptr) {
      mem_unreserve(dev, size, kDeviceBuf);
      return rc;
    }
    ledger_add(*ptr, size, dev, kDeviceBuf);
    return rc;
  }
  hsa_status_t rc = real(pool, size, flags, ptr);
  if (rc != HSA_STATUS_SUCCESS || !ptr || !*ptr) return rc;
  mem_charge_nofail(dev, size, kRuntime);
  ledger_add(*ptr, size, dev, kRuntime);
  return rc;
}

hsa_status_t pool_free_impl(decltype(&::hsa_amd_memory_pool_free) real, void* ptr) {
  Alloc a;
  if (ptr && (ledger_take_if(ptr, kRuntime, &a) || ledger_take_if(ptr, kDeviceBuf, &a)))
    mem_unreserve(a.dev, a.size, a.kind);
  return real(ptr);
}

// ---- dispatch interception below HIP (VERDICT r4 missing #4) ---------------------------
// The reference catches every kernel at cuLaunchKernel, CUDA's one driver entry
// point.  HIP's launches are caught by the HIP hooks; a library that dispatches
// AQL packets on HSA queues of its own bypasses them.  ROCr exports no
// intercept-queue symbols, but its tools API table carries
// hsa_amd_queue_intercept_create / _register (the rocprofiler mechanism), so in
// table mode (HSA_TOOLS_LIB=libvgpu.so) a queue the HIP runtime did not create
// becomes an intercept queue: every batch of packets written to it reaches
// dispatch_handler before the hardware ring.  Its kernel dispatches are counted
// (workgroups from the packet's grid / workgroup sizes) and pass the same gate
// as a HIP launch -- suspend, task priority, the temporal limiter's hold -- and
// their busy time is charged by the KFD cu_occupancy cross-check (occ_step),
// which charges what no marker covers.  VGPU_HSA_DISPATCH=auto (default) /
// all (HIP's queues too, counted only: the HIP hooks already gate those) / off.
struct QInfo {
  int dev;
  bool hip;  // created by the HIP runtime: count, never gate twice
};

int dispatch_mode() {  // 0 off, 1 auto, 2 all
  static const int m = [] {
    const char* v = env_first("VGPU_HSA_DISPATCH");
    if (!v || !*v || !strcasecmp(v, "auto")) return 1;
    if (!strcasecmp(v, "all")) return 2;
    return env_bool(v, true) ? 1 : 0;
  }();
  return m;
}

// The HIP runtime (ROCclr lives in libamdhip64) on the stack of this queue
// creation?  Queue creation is rare: a backtrace is cheap enough.
bool created_by_hip() {
  void* frames[24];
  const int n = backtrace(frames, 24);
  for (int i = 0; i < n; ++i) {
    Dl_info di;
    if (dladdr(frames[i], &di) && di.dli_fname && strstr(di.dli_fname, "libamdhip64")) return true;
  }
  return false;
}

void dispatch_handler(const void* pkts, uint64_t n, uint64_t, void* data,
                      hsa_amd_queue_intercept_packet_writer writer) {
  const auto* qi = static_cast<const QInfo*>(data);
  const auto* p = static_cast<const hsa_kernel_dispatch_packet_t*>(pkts);
  uint64_t wg = 0;
  uint32_t kernels = 0;
  for (uint64_t i = 0; i < n; ++i) {
    if ((p[i].header & 0xff) != HSA_PACKET_TYPE_KERNEL_DISPATCH) continue;
    auto blocks = [](uint32_t g, uint16_t w) -> uint64_t { return w ? (g + w - 1) / w : g; };
    wg += blocks(p[i].grid_size_x, p[i].workgroup_size_x) * blocks(p[i].grid_size_y, p[i].workgroup_size_y) *
          blocks(p[i].grid_size_z, p[i].workgroup_size_z);
    ++kernels;
  }
  if (kernels) {
    g_hsa_dispatches.fetch_add(kernels, std::memory_order_relaxed);
    if (qi && !qi->hip) (void)limiter_on_launch(qi->dev, wg, nullptr, kernels);
  }
  writer(pkts, n);
}

// Table entries (HSA_TOOLS_LIB mode).
hsa_status_t tab_queue_create(hsa_agent_t agent, uint32_t size, hsa_queue_type32_t type,
                              void (*cb)(hsa_status_t, hsa_queue_t*, void*), void* data,
                              uint32_t priv, uint32_t group, hsa_queue_t** queue) {
  ensure_init();
  const int mode = dispatch_mode();
  if (mode && g_orig.intercept_create && g_orig.intercept_register && st().enabled) {
    const bool hip = created_by_hip();
    const int dev = cumask_hip_index_for_agent(agent.handle);
    if (dev >= 0 && (mode == 2 || !hip)) {
      hsa_status_t rc = queue_create_impl(g_orig.intercept_create, agent, size, type, cb, data, priv, group, queue);
      if (rc != HSA_STATUS_SUCCESS) return rc;
      auto* qi = new QInfo{dev, hip};  // lives as long as the process (queues are few)
      if (g_orig.intercept_register(*queue, dispatch_handler, qi) == HSA_STATUS_SUCCESS) {
        g_hsa_intercepted_queues.fetch_add(1);
        VLOG_INFO("device %d queue %p: dispatches intercepted (%s queue)", dev, (void*)*queue,
                  hip ? "HIP" : "non-HIP");
      } else {
        VLOG_WARN("device %d queue %p: intercept registration failed; dispatches not gated", dev, (void*)*queue);
      }
      return rc;
    }
  }
  return queue_create_impl(g_orig.queue_create, agent, size, type, cb, data, priv, group, queue);
}
hsa_status_t tab_queue_destroy(hsa_queue_t* queue) {
  cumask_on_queue_destroyed(queue);
  return g_orig.queue_destroy(queue);
}
hsa_status_t tab_cu_set_mask(const hsa_queue_t* q, uint32_t n, const uint32_t* m) {
  return cu_set_mask_impl(g_orig.cu_set_mask, q, n, m);
}
hsa_status_t tab_pool_allocate(hsa_amd_memory_pool_t pool, size_t size, uint32_t flags, void** ptr) {
  const void* caller = tl_pool_caller;
  tl_pool_caller = nullptr;
  return pool_allocate_impl(g_orig.pool_allocate, pool, size, flags, ptr, caller);
}
hsa_status_t tab_pool_free(void* ptr) { return pool_free_impl(g_orig.pool_free, ptr); }

}  // namespace

bool hsa_table_mode() { return g_table_mode.load(std::memory_order_acquire); }

// The runtime's own cu_set_mask, for the shim's internal use: in table mode the
// exported symbol would come back through tab_cu_set_mask (and its lock).
hsa_status_t real_cu_set_mask(const hsa_queue_t* q, uint32_t bits, const uint32_t* mask) {
  if (hsa_table_mode()) return g_orig.cu_set_mask(q, bits, mask);
  return REAL_HSA(hsa_amd_queue_cu_set_mask)(q, bits, mask);
}

}  // namespace vgpu

using namespace vgpu;

extern "C" {

__attribute__((visibility("default"))) hsa_status_t hsa_queue_create(
    hsa_agent_t agent, uint32_t size, hsa_queue_type32_t type,
    void (*callback)(hsa_status_t status, hsa_queue_t* source, void* data), void* data,
    uint32_t private_segment_size, uint32_t group_segment_size, hsa_queue_t** queue) {
  if (hsa_table_mode())
    return REAL_HSA(hsa_queue_create)(agent, size, type, callback, data, private_segment_size,
                                      group_segment_size, queue);
  return queue_create_impl(REAL_HSA(hsa_queue_create), agent, size, type, callback, data,
                           private_segment_size, group_segment_size, queue);
}

__attribute__((visibility("default"))) hsa_status_t hsa_queue_destroy(hsa_queue_t* queue) {
  if (!hsa_table_mode()) cumask_on_queue_destroyed(queue);
  return REAL_HSA(hsa_queue_destroy)(queue);
}

__attribute__((visibility("default"))) hsa_status_t hsa_amd_queue_cu_set_mask(
    const hsa_queue_t* queue, uint32_t num_cu_mask_count, const uint32_t* cu_mask) {
  if (hsa_table_mode()) return REAL_HSA(hsa_amd_queue_cu_set_mask)(queue, num_cu_mask_count, cu_mask);
  return cu_set_mask_impl(REAL_HSA(hsa_amd_queue_cu_set_mask), queue, num_cu_mask_count, cu_mask);
}

__attribute__((visibility("default"))) hsa_status_t hsa_amd_memory_pool_allocate(
    hsa_amd_memory_pool_t pool, size_t size, uint32_t flags, void** ptr) {
  const void* caller = __builtin_return_address(0);
  if (hsa_table_mode()) {
    tl_pool_caller = caller;  // the table entry runs next, on this thread
    hsa_status_t rc = REAL_HSA(hsa_amd_memory_pool_allocate)(pool, size, flags, ptr);
    tl_pool_caller = nullptr;
    return rc;
  }
  return pool_allocate_impl(REAL_HSA(hsa_amd_memory_pool_allocate), pool, size, flags, ptr, caller);
}

__attribute__((visibility("default"))) hsa_status_t hsa_amd_memory_pool_free(void* ptr) {
  if (hsa_table_mode()) return REAL_HSA(hsa_amd_memory_pool_free)(ptr);
  return pool_free_impl(REAL_HSA(hsa_amd_memory_pool_free), ptr);
}

// ROCr tools-library entry (HSA_TOOLS_LIB).  Runs inside hsa_init, before any
// queue or pool allocation of the process.
__attribute__((visibility("default"))) bool OnLoad(void* api_table, uint64_t runtime_version,
                                                   uint64_t failed_tool_count,
                                                   const char* const* failed_tool_names) {
  auto* t = static_cast<HsaApiTable*>(api_table);
  if (!t || !t->core_ || !t->amd_ext_) return true;
  g_orig.queue_create = t->core_->hsa_queue_create_fn;
  g_orig.queue_destroy = t->core_->hsa_queue_destroy_fn;
  g_orig.cu_set_mask = t->amd_ext_->hsa_amd_queue_cu_set_mask_fn;
  g_orig.pool_allocate = t->amd_ext_->hsa_amd_memory_pool_allocate_fn;
  g_orig.pool_free = t->amd_ext_->hsa_amd_memory_pool_free_fn;
  g_orig.intercept_create = t->amd_ext_->hsa_amd_queue_intercept_create_fn;
  g_orig.intercept_register = t->amd_ext_->hsa_amd_queue_intercept_register_fn;
  if (!g_orig.queue_create || !g_orig.queue_destroy || !g_orig.cu_set_mask ||
      !g_orig.pool_allocate || !g_orig.pool_free)
    return true;  // unknown table layout: stay on the PLT interposers
  t->core_->hsa_queue_create_fn = tab_queue_create;
  t->core_->hsa_queue_destroy_fn = tab_queue_destroy;
  t->amd_ext_->hsa_amd_queue_cu_set_mask_fn = tab_cu_set_mask;
  t->amd_ext_->hsa_amd_memory_pool_allocate_fn = tab_pool_allocate;
  t->amd_ext_->hsa_amd_memory_pool_free_fn = tab_pool_free;
  g_table_mode.store(true, std::memory_order_release);
  VLOG_INFO("HSA API table intercepted (runtime %llu)", (unsigned long long)runtime_version);
  return true;
}

__attribute__((visibility("default"))) void OnUnload() {}

}  // extern "C"
