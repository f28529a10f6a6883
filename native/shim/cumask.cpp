// Spatial compute partitioning: XCD-balanced CU masks on every HSA queue.
//
// Reference analogue: the Hygon DCU plugin writes a `cu_mask` hex string into a
// per-container vdev file consumed by the vendor driver
// (pkg/device-plugin/hygon/dcu/server.go:415-459, corealloc.go:60-77); the
// NVIDIA path has no spatial partitioning at all (token bucket only).
//
// MI355X: ROCr exposes hsa_amd_queue_cu_set_mask().  Every queue the HIP
// runtime creates (hsa_queue_create, hooked in hooks_hsa.cpp) gets the
// container's mask, so every dispatch from the process — PyTorch kernels,
// hipBLASLt / MIOpen / RCCL internals, hipGraph replays — is confined to its
// CUs with zero per-dispatch cost.
//
// Mask bit semantics on multi-XCD gfx950 (verified on MI355X by
// tests/test_gpu_shim.py::test_cu_mask_census): logical bit i is mapped to XCD
// (i % num_xcc), so any contiguous run of 8k low-order logical bits gives every
// XCD k CUs — the allocator in vgpu/device/cualloc.py hands out masks in
// such 8-bit granules.  VGPU_CU_MASK_LAYOUT=blocked switches to the
// bit i -> XCD (i / cus_per_xcc) interpretation.
#include <algorithm>
#include <vector>

#include "common.h"
#include "real.h"
#include "state.h"

namespace vgpu {

struct AgentInfo {
  hsa_agent_t agent;
  uint32_t cus = 0;
  uint32_t num_xcc = 1;
  uint32_t driver_uid = 0;
  int hip_index = -1;  // device ordinal as seen by HIP (after HIP_VISIBLE_DEVICES)
};

static std::mutex g_mu;
static std::vector<AgentInfo> g_agents;
static bool g_agents_ready = false;
static std::vector<std::pair<hsa_queue_t*, int>> g_queues;  // queue, hip device

static hsa_status_t collect_agent(hsa_agent_t a, void* data) {
  auto* v = (std::vector<AgentInfo>*)data;
  hsa_device_type_t t;
  if (REAL_HSA(hsa_agent_get_info)(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (t != HSA_DEVICE_TYPE_GPU) return HSA_STATUS_SUCCESS;
  AgentInfo ai;
  ai.agent = a;
  REAL_HSA(hsa_agent_get_info)(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_COMPUTE_UNIT_COUNT, &ai.cus);
  uint32_t nx = 0;
  if (REAL_HSA(hsa_agent_get_info)(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_NUM_XCC, &nx) == HSA_STATUS_SUCCESS && nx)
    ai.num_xcc = nx;
  REAL_HSA(hsa_agent_get_info)(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DRIVER_UID, &ai.driver_uid);
  v->push_back(ai);
  return HSA_STATUS_SUCCESS;
}

static std::vector<int> visible_list() {
  std::vector<int> out;
  const char* v = env_first("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES");
  if (!v) return out;
  const char* p = v;
  while (*p) {
    char* end;
    long x = strtol(p, &end, 10);
    if (end == p) return {};  // UUID-style list: treat as identity
    out.push_back((int)x);
    p = end;
    while (*p == ',' || *p == ' ') ++p;
  }
  return out;
}

static void ensure_agents_locked() {
  if (g_agents_ready) return;
  std::vector<AgentInfo> v;
  if (REAL_HSA(hsa_iterate_agents)(collect_agent, &v) != HSA_STATUS_SUCCESS) return;
  std::vector<int> vis = visible_list();
  for (size_t a = 0; a < v.size(); ++a) {
    if (vis.empty()) {
      v[a].hip_index = (int)a;
    } else {
      auto it = std::find(vis.begin(), vis.end(), (int)a);
      v[a].hip_index = it == vis.end() ? -1 : (int)(it - vis.begin());
    }
  }
  g_agents = v;
  g_agents_ready = true;
}

static AgentInfo* agent_for_hip_index(int dev) {
  for (auto& a : g_agents)
    if (a.hip_index == dev) return &a;
  return nullptr;
}

static bool mask_for_device(int dev, const AgentInfo& ai, uint64_t out[VGPU_CU_MASK_WORDS]) {
  State& s = st();
  memset(out, 0, sizeof(uint64_t) * VGPU_CU_MASK_WORDS);
  if (!s.enabled || dev < 0 || dev >= VGPU_MAX_DEVICES || s.lim.core_policy == 2) return false;
  bool has = false;
  if (s.region) {
    for (int w = 0; w < VGPU_CU_MASK_WORDS; ++w) {
      out[w] = __atomic_load_n(&s.region->dev[dev].cu_mask[w], __ATOMIC_RELAXED);
      has |= out[w] != 0;
    }
  }
  if (has) return true;
  uint32_t lim = s.region ? s.region->dev[dev].cu_limit : s.lim.cu_limit[dev];
  if (lim == 0 || lim >= 100 || !env_bool(env_first("VGPU_CU_MASK_FROM_LIMIT"), true)) return false;
  // Derive a balanced mask: ceil(lim% of CUs) rounded up to whole granules of
  // one CU per XCD, taken from the low logical bits.
  uint32_t cus = ai.cus ? ai.cus : 256;
  uint32_t nx = ai.num_xcc ? ai.num_xcc : 1;
  uint32_t n = (cus * lim + 99) / 100;
  n = ((n + nx - 1) / nx) * nx;
  if (n > cus) n = cus;
  const char* layout = env_first("VGPU_CU_MASK_LAYOUT");
  bool blocked = layout && !strcasecmp(layout, "blocked");
  uint32_t per = cus / nx;
  for (uint32_t k = 0; k < n; ++k) {
    uint32_t bit = blocked ? (k % nx) * per + (k / nx) : k;
    if (bit < VGPU_CU_MASK_WORDS * 64) out[bit / 64] |= 1ull << (bit % 64);
  }
  return true;
}

static void apply_mask(hsa_queue_t* q, int dev, const AgentInfo& ai) {
  uint64_t m[VGPU_CU_MASK_WORDS];
  if (!mask_for_device(dev, ai, m)) return;
  uint32_t cus = ai.cus ? ai.cus : 256;
  uint32_t bits = ((cus + 31) / 32) * 32;
  if (bits > VGPU_CU_MASK_WORDS * 64) bits = VGPU_CU_MASK_WORDS * 64;
  uint32_t words32[VGPU_CU_MASK_WORDS * 2];
  for (int w = 0; w < VGPU_CU_MASK_WORDS; ++w) {
    words32[2 * w] = (uint32_t)(m[w] & 0xffffffffu);
    words32[2 * w + 1] = (uint32_t)(m[w] >> 32);
  }
  hsa_status_t rc = real_cu_set_mask(q, bits, words32);
  if (rc != HSA_STATUS_SUCCESS && (int)rc != (int)HSA_STATUS_CU_MASK_REDUCED) {
    VLOG_WARN("hsa_amd_queue_cu_set_mask failed on device %d: %d", dev, (int)rc);
  } else {
    VLOG_INFO("device %d queue %p: CU mask %s", dev, (void*)q,
              format_cu_mask(m, VGPU_CU_MASK_WORDS).c_str());
    int n = 0;
    for (int w = 0; w < VGPU_CU_MASK_WORDS; ++w) n += __builtin_popcountll(m[w]);
    trace_emit(VGPU_EV_QUEUE, dev, (uint64_t)(uintptr_t)q, (uint64_t)n);
  }
}

int cumask_hip_index_for_agent(uint64_t agent_handle) {
  std::lock_guard<std::mutex> g(g_mu);
  ensure_agents_locked();
  for (auto& a : g_agents)
    if (a.agent.handle == agent_handle) return a.hip_index;
  return -1;
}

void cumask_on_queue_created(void* agent_ptr, void* queue) {
  State& s = st();
  if (!s.enabled) return;
  hsa_agent_t agent = *(hsa_agent_t*)agent_ptr;
  std::lock_guard<std::mutex> g(g_mu);
  ensure_agents_locked();
  for (auto& a : g_agents) {
    if (a.agent.handle != agent.handle) continue;
    if (a.hip_index < 0) return;
    g_queues.push_back({(hsa_queue_t*)queue, a.hip_index});
    apply_mask((hsa_queue_t*)queue, a.hip_index, a);
    return;
  }
}

void cumask_on_queue_destroyed(void* queue) {
  std::lock_guard<std::mutex> g(g_mu);
  g_queues.erase(std::remove_if(g_queues.begin(), g_queues.end(),
                                [&](const std::pair<hsa_queue_t*, int>& e) {
                                  return e.first == (hsa_queue_t*)queue;
                                }),
                 g_queues.end());
}

int cumask_reapply_all() {
  std::lock_guard<std::mutex> g(g_mu);
  int n = 0;
  for (auto& q : g_queues) {
    AgentInfo* a = agent_for_hip_index(q.second);
    if (!a) continue;
    uint64_t m[VGPU_CU_MASK_WORDS];
    if (mask_for_device(q.second, *a, m)) {
      apply_mask(q.first, q.second, *a);
    } else {
      // Back to every CU: an explicit all-ones mask.  A zero-length mask is not
      // a reset (ROCr leaves the queue on its previous CUs), which kept an
      // auto pod on its spatial claim through the time-shared window after it
      // (profiles/r4: the A/B/A windows disagreed 554 vs 297 dispatches/s).
      const uint32_t cus = a->cus ? a->cus : 256;
      const uint32_t bits = std::min<uint32_t>(((cus + 31) / 32) * 32, VGPU_CU_MASK_WORDS * 64);
      uint32_t words32[VGPU_CU_MASK_WORDS * 2];
      for (uint32_t i = 0; i < VGPU_CU_MASK_WORDS * 2; ++i) {
        const uint32_t lo = 32 * i;
        words32[i] = cus <= lo ? 0u : (cus >= lo + 32 ? ~0u : ((1u << (cus - lo)) - 1));
      }
      const hsa_status_t rc = real_cu_set_mask(q.first, bits, words32);
      if (rc != HSA_STATUS_SUCCESS && (int)rc != (int)HSA_STATUS_CU_MASK_REDUCED)
        VLOG_WARN("hsa_amd_queue_cu_set_mask (all CUs) failed on device %d: %d", q.second, (int)rc);
      else
        VLOG_INFO("device %d queue %p: CU mask reset to all %u CUs", q.second, (void*)q.first, cus);
      trace_emit(VGPU_EV_QUEUE, q.second, (uint64_t)(uintptr_t)q.first, (uint64_t)cus);
    }
    ++n;
  }
  return n;
}

// Intersect an application-requested mask with the container's mask.
bool cumask_intersect(const hsa_queue_t* q, uint32_t* bits, const uint32_t* in, uint32_t* out) {
  std::lock_guard<std::mutex> g(g_mu);
  for (auto& e : g_queues) {
    if (e.first != q) continue;
    AgentInfo* a = agent_for_hip_index(e.second);
    if (!a) return false;
    uint64_t m[VGPU_CU_MASK_WORDS];
    if (!mask_for_device(e.second, *a, m)) return false;
    uint32_t n = *bits;
    if (n == 0) {  // "all CUs" request → our mask
      n = ((a->cus ? a->cus : 256) + 31) / 32 * 32;
      for (uint32_t w = 0; w < n / 32; ++w)
        out[w] = (uint32_t)(m[w / 2] >> (32 * (w % 2)));
    } else {
      for (uint32_t w = 0; w < n / 32 && w < VGPU_CU_MASK_WORDS * 2; ++w)
        out[w] = in[w] & (uint32_t)(m[w / 2] >> (32 * (w % 2)));
    }
    *bits = n;
    return true;
  }
  return false;
}

int cumask_device_cus(int dev) {
  std::lock_guard<std::mutex> g(g_mu);
  ensure_agents_locked();
  AgentInfo* a = agent_for_hip_index(dev);
  if (!a) return -1;
  uint64_t m[VGPU_CU_MASK_WORDS];
  if (mask_for_device(dev, *a, m)) {
    int n = 0;
    for (int w = 0; w < VGPU_CU_MASK_WORDS; ++w) n += __builtin_popcountll(m[w]);
    return n;
  }
  return (int)a->cus;
}

int cumask_device_physical_cus(int dev) {
  std::lock_guard<std::mutex> g(g_mu);
  ensure_agents_locked();
  AgentInfo* a = agent_for_hip_index(dev);
  return a ? (int)a->cus : -1;
}

bool hsa_gpu_agent(int dev, hsa_agent_t* out) {
  std::lock_guard<std::mutex> g(g_mu);
  ensure_agents_locked();
  AgentInfo* a = agent_for_hip_index(dev);
  if (!a) return false;
  *out = a->agent;
  return true;
}

bool hsa_cpu_agent(hsa_agent_t* out) {
  static hsa_agent_t cpu{0};
  static std::once_flag once;
  std::call_once(once, [] {
    REAL_HSA(hsa_iterate_agents)([](hsa_agent_t a, void* d) {
      hsa_device_type_t t;
      if (REAL_HSA(hsa_agent_get_info)(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
        *(hsa_agent_t*)d = a;
        return HSA_STATUS_INFO_BREAK;
      }
      return HSA_STATUS_SUCCESS;
    }, &cpu);
  });
  *out = cpu;
  return cpu.handle != 0;
}

uint32_t cumask_driver_uid(int dev) {
  std::lock_guard<std::mutex> g(g_mu);
  AgentInfo* a = agent_for_hip_index(dev);
  return a ? a->driver_uid : 0;
}

// Device-memory pools (GLOBAL segment) of every container-visible GPU agent,
// for the HSA pool-allocation accounting in hooks_hsa.cpp.
static std::vector<std::pair<uint64_t, int>> g_pools;  // pool handle, hip device
static bool g_pools_ready = false;

static hsa_status_t collect_pool(hsa_amd_memory_pool_t pool, void* data) {
  auto* out = static_cast<std::vector<uint64_t>*>(data);
  hsa_amd_segment_t seg;
  if (REAL_HSA(hsa_amd_memory_pool_get_info)(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) ==
          HSA_STATUS_SUCCESS &&
      seg == HSA_AMD_SEGMENT_GLOBAL)
    out->push_back(pool.handle);
  return HSA_STATUS_SUCCESS;
}

int cumask_hip_index_for_pool(uint64_t pool_handle) {
  std::lock_guard<std::mutex> g(g_mu);
  if (!g_pools_ready) {
    ensure_agents_locked();
    if (!g_agents_ready) return -1;
    for (auto& a : g_agents) {
      if (a.hip_index < 0) continue;
      std::vector<uint64_t> pools;
      REAL_HSA(hsa_amd_agent_iterate_memory_pools)(a.agent, collect_pool, &pools);
      for (uint64_t p : pools) g_pools.push_back({p, a.hip_index});
    }
    g_pools_ready = true;
  }
  for (auto& e : g_pools)
    if (e.first == pool_handle) return e.second;
  return -1;
}

int cu_count_masked(int dev, int physical) {
  int n = cumask_device_cus(dev);
  if (n <= 0 || n > physical) return physical;
  return n;
}

}  // namespace vgpu
