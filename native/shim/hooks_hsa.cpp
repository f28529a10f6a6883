// ROCr (HSA) interposers: catch every hardware queue the process creates so the
// container's CU mask is applied before the first dispatch, and keep the
// application from widening it.
//
// This has no reference counterpart (CUDA offers no per-stream SM mask); it is
// the MI355X replacement for the time-sliced SM limiter (SURVEY.md §2.6 E1f,
// §7.2 step 3(a)).
#include "common.h"
#include "real.h"
#include "state.h"

namespace vgpu {
bool cumask_intersect(const hsa_queue_t* q, uint32_t* bits, const uint32_t* in, uint32_t* out);
}

using namespace vgpu;

extern "C" {

__attribute__((visibility("default"))) hsa_status_t hsa_queue_create(
    hsa_agent_t agent, uint32_t size, hsa_queue_type32_t type,
    void (*callback)(hsa_status_t status, hsa_queue_t* source, void* data), void* data,
    uint32_t private_segment_size, uint32_t group_segment_size, hsa_queue_t** queue) {
  ensure_init();
  hsa_status_t rc = REAL_HSA(hsa_queue_create)(agent, size, type, callback, data,
                                               private_segment_size, group_segment_size, queue);
  if (rc == HSA_STATUS_SUCCESS && queue && *queue) cumask_on_queue_created(&agent, *queue);
  return rc;
}

__attribute__((visibility("default"))) hsa_status_t hsa_queue_destroy(hsa_queue_t* queue) {
  cumask_on_queue_destroyed(queue);
  return REAL_HSA(hsa_queue_destroy)(queue);
}

__attribute__((visibility("default"))) hsa_status_t hsa_amd_queue_cu_set_mask(
    const hsa_queue_t* queue, uint32_t num_cu_mask_count, const uint32_t* cu_mask) {
  ensure_init();
  uint32_t bits = num_cu_mask_count;
  uint32_t merged[VGPU_CU_MASK_WORDS * 2] = {};
  if (num_cu_mask_count <= VGPU_CU_MASK_WORDS * 64 &&
      cumask_intersect(queue, &bits, cu_mask, merged))
    return REAL_HSA(hsa_amd_queue_cu_set_mask)(queue, bits, merged);
  return REAL_HSA(hsa_amd_queue_cu_set_mask)(queue, num_cu_mask_count, cu_mask);
}

}  // extern "C"
