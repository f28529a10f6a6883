// amdsmi / rocm-smi memory virtualisation: inside a vGPU container, `amd-smi`,
// `rocm-smi`, and PyTorch's amdsmi queries report the container's HBM cap as
// the device's VRAM and the container's usage as "used".
//
// Reference behaviour: libvgpu.so hooks 247 nvml* entry points; the ones with
// behaviour are nvmlDeviceGetMemoryInfo (1190 B) / _v2 (1214 B), which report
// the container's limit and usage, everything else passes through
// (SURVEY.md §2.6 E1c).  The MI355X equivalents are amdsmi_get_gpu_memory_total
// / _usage, amdsmi_get_gpu_vram_usage / _info (libamd_smi) and
// rsmi_dev_memory_total_get / _usage_get (librocm_smi64).  Lookups made by
// ctypes through a dlopen handle reach these via the dlsym interposer
// (dlsym.cpp).
//
// Process lists (reference: NVML process-list virtualisation, §2.6 E1c) are
// filtered to this container's processes: the host pids of its region's slots
// as resolved by hostpid.cpp.  A process whose host pid is unknown is hidden
// rather than guessed.
//
// Device index: the limit arrays are indexed by the container's visible device
// ordinal.  Inside a pod only the allocated GPUs' render nodes exist, and
// amdsmi / rocm-smi enumerate them in the same (KFD node) order HIP does.
#include <amd_smi/amdsmi.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "common.h"
#include "real.h"
#include "state.h"

using namespace vgpu;

namespace {

#define REAL_SMI(name) \
  ((decltype(&::name))smi_real(#name, __builtin_return_address(0), amdsmi_lib_handle))

std::mutex g_mu;
std::vector<amdsmi_processor_handle> g_gpus;
bool g_ready = false;

int gpu_index(amdsmi_processor_handle h) {
  std::lock_guard<std::mutex> g(g_mu);
  if (!g_ready) {
    uint32_t ns = 0;
    if (REAL_SMI(amdsmi_get_socket_handles)(&ns, nullptr) == AMDSMI_STATUS_SUCCESS && ns) {
      std::vector<amdsmi_socket_handle> socks(ns);
      if (REAL_SMI(amdsmi_get_socket_handles)(&ns, socks.data()) == AMDSMI_STATUS_SUCCESS) {
        for (uint32_t s = 0; s < ns; ++s) {
          uint32_t np = 0;
          if (REAL_SMI(amdsmi_get_processor_handles)(socks[s], &np, nullptr) != AMDSMI_STATUS_SUCCESS)
            continue;
          std::vector<amdsmi_processor_handle> ps(np);
          if (REAL_SMI(amdsmi_get_processor_handles)(socks[s], &np, ps.data()) != AMDSMI_STATUS_SUCCESS)
            continue;
          for (uint32_t i = 0; i < np; ++i) {
            processor_type_t t = AMDSMI_PROCESSOR_TYPE_UNKNOWN;
            if (REAL_SMI(amdsmi_get_processor_type)(ps[i], &t) == AMDSMI_STATUS_SUCCESS &&
                t == AMDSMI_PROCESSOR_TYPE_AMD_GPU)
              g_gpus.push_back(ps[i]);
          }
        }
      }
    }
    g_ready = !g_gpus.empty();
  }
  auto it = std::find(g_gpus.begin(), g_gpus.end(), h);
  return it == g_gpus.end() ? -1 : (int)(it - g_gpus.begin());
}

bool is_vram(amdsmi_memory_type_t t) {
  return t == AMDSMI_MEM_TYPE_VRAM || t == AMDSMI_MEM_TYPE_VIS_VRAM;
}

// Container limit of the device behind `h` (0 = not virtualised).
uint64_t limit_of(amdsmi_processor_handle h, int* dev_out) {
  ensure_init();
  if (!st().enabled) return 0;
  int dev = gpu_index(h);
  if (dev_out) *dev_out = dev;
  return dev < 0 ? 0 : mem_limit(dev);
}

uint64_t hbm_used(int dev) {
  State& s = st();
  return s.region ? region_device_used(s.region, dev) : 0;
}

}  // namespace

extern "C" {

__attribute__((visibility("default"))) amdsmi_status_t amdsmi_get_gpu_memory_total(
    amdsmi_processor_handle h, amdsmi_memory_type_t type, uint64_t* total) {
  amdsmi_status_t rc = REAL_SMI(amdsmi_get_gpu_memory_total)(h, type, total);
  if (rc != AMDSMI_STATUS_SUCCESS || !total || !is_vram(type)) return rc;
  if (uint64_t lim = limit_of(h, nullptr)) *total = lim;
  return rc;
}

__attribute__((visibility("default"))) amdsmi_status_t amdsmi_get_gpu_memory_usage(
    amdsmi_processor_handle h, amdsmi_memory_type_t type, uint64_t* used) {
  amdsmi_status_t rc = REAL_SMI(amdsmi_get_gpu_memory_usage)(h, type, used);
  if (rc != AMDSMI_STATUS_SUCCESS || !used || !is_vram(type)) return rc;
  int dev = -1;
  if (uint64_t lim = limit_of(h, &dev)) *used = std::min<uint64_t>(hbm_used(dev), lim);
  return rc;
}

__attribute__((visibility("default"))) amdsmi_status_t amdsmi_get_gpu_vram_usage(
    amdsmi_processor_handle h, amdsmi_vram_usage_t* info) {
  amdsmi_status_t rc = REAL_SMI(amdsmi_get_gpu_vram_usage)(h, info);
  if (rc != AMDSMI_STATUS_SUCCESS || !info) return rc;
  int dev = -1;
  if (uint64_t lim = limit_of(h, &dev)) {
    info->vram_total = (uint32_t)(lim >> 20);
    info->vram_used = (uint32_t)(std::min<uint64_t>(hbm_used(dev), lim) >> 20);
  }
  return rc;
}

__attribute__((visibility("default"))) amdsmi_status_t amdsmi_get_gpu_process_list(
    amdsmi_processor_handle h, uint32_t* max, amdsmi_proc_info_t* list) {
  auto real = REAL_SMI(amdsmi_get_gpu_process_list);
  ensure_init();
  if (!st().enabled || !max) return real(h, max, list);
  // Fetch the whole device list, then keep only our own processes.
  uint32_t n = 0;
  amdsmi_status_t rc = real(h, &n, nullptr);
  if (rc != AMDSMI_STATUS_SUCCESS && rc != AMDSMI_STATUS_OUT_OF_RESOURCES) return rc;
  std::vector<amdsmi_proc_info_t> all(n + 16);
  uint32_t got = (uint32_t)all.size();
  rc = real(h, &got, all.data());
  if (rc != AMDSMI_STATUS_SUCCESS) return rc;
  const std::vector<int> mine = container_host_pids();
  uint32_t k = 0;
  const uint32_t cap = list ? *max : 0;
  for (uint32_t i = 0; i < got && i < all.size(); ++i) {
    if (std::find(mine.begin(), mine.end(), (int)all[i].pid) == mine.end()) continue;
    if (k < cap) list[k] = all[i];
    ++k;
  }
  *max = k;
  return AMDSMI_STATUS_SUCCESS;
}

__attribute__((visibility("default"))) amdsmi_status_t amdsmi_get_gpu_vram_info(
    amdsmi_processor_handle h, amdsmi_vram_info_t* info) {
  amdsmi_status_t rc = REAL_SMI(amdsmi_get_gpu_vram_info)(h, info);
  if (rc != AMDSMI_STATUS_SUCCESS || !info) return rc;
  if (uint64_t lim = limit_of(h, nullptr)) info->vram_size = lim >> 20;
  return rc;
}

}  // extern "C"
