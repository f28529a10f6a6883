// rocm-smi (librocm_smi64) memory virtualisation — the rocm-smi twin of
// hooks_smi.cpp (reference: nvmlDeviceGetMemoryInfo).
// rsmi device indices are the container-visible ordinals.
#include <rocm_smi/rocm_smi.h>

#include <algorithm>

#include "common.h"
#include "real.h"
#include "state.h"

using namespace vgpu;

#define REAL_RSMI(name) \
  ((decltype(&::name))smi_real(#name, __builtin_return_address(0), rsmi_lib_handle))

static bool rsmi_vram(rsmi_memory_type_t t) {
  return t == RSMI_MEM_TYPE_VRAM || t == RSMI_MEM_TYPE_VIS_VRAM;
}

static uint64_t rsmi_limit(uint32_t dv) {
  ensure_init();
  if (!st().enabled || dv >= VGPU_MAX_DEVICES) return 0;
  return mem_limit((int)dv);
}

extern "C" {

__attribute__((visibility("default"))) rsmi_status_t rsmi_dev_memory_total_get(
    uint32_t dv_ind, rsmi_memory_type_t type, uint64_t* total) {
  rsmi_status_t rc = REAL_RSMI(rsmi_dev_memory_total_get)(dv_ind, type, total);
  if (rc != RSMI_STATUS_SUCCESS || !total || !rsmi_vram(type)) return rc;
  if (uint64_t lim = rsmi_limit(dv_ind)) *total = lim;
  return rc;
}

__attribute__((visibility("default"))) rsmi_status_t rsmi_dev_memory_usage_get(
    uint32_t dv_ind, rsmi_memory_type_t type, uint64_t* used) {
  rsmi_status_t rc = REAL_RSMI(rsmi_dev_memory_usage_get)(dv_ind, type, used);
  if (rc != RSMI_STATUS_SUCCESS || !used || !rsmi_vram(type)) return rc;
  if (uint64_t lim = rsmi_limit(dv_ind)) {
    State& s = st();
    uint64_t u = s.region ? region_device_used(s.region, (int)dv_ind) : 0;
    *used = std::min<uint64_t>(u, lim);
  }
  return rc;
}

}  // extern "C"
