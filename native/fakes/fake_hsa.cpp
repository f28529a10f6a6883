// JSON/env-driven fake of the ROCr (HSA) runtime, for CPU-only tests of the
// enforcement library.  Mirrors the role of the reference's fake libcndev.so
// (pkg/device-plugin/mlu/cndev/mock/cndev.c:22-39): a real shared object with
// the vendor ABI, answering from a fixture instead of hardware.
//
// Built as libhsa-runtime64.so.1 (SONAME) with the ROCR_1 symbol version.
// Fixture: VGPU_FAKE_GPUS (default 1), VGPU_FAKE_CUS (256), VGPU_FAKE_XCC (8).
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <vector>

namespace {

struct FakeQueue {
  hsa_queue_t q;
  uint64_t agent;
  uint32_t mask[8];
  uint32_t mask_bits;
  int alive;
};

std::mutex g_mu;
std::vector<FakeQueue*> g_queues;

int env_int(const char* n, int d) {
  const char* v = getenv(n);
  return v && *v ? atoi(v) : d;
}

}  // namespace

extern "C" {

hsa_status_t hsa_init() { return HSA_STATUS_SUCCESS; }
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

hsa_status_t hsa_queue_create(hsa_agent_t agent, uint32_t size, hsa_queue_type32_t type,
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

hsa_status_t hsa_queue_destroy(hsa_queue_t* q) {
  std::lock_guard<std::mutex> g(g_mu);
  for (auto* fq : g_queues)
    if (&fq->q == q) fq->alive = 0;
  return HSA_STATUS_SUCCESS;
}

hsa_status_t hsa_amd_queue_cu_set_mask(const hsa_queue_t* q, uint32_t bits, const uint32_t* mask) {
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

// ---- test introspection ----
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
