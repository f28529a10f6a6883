// rocm-smi (librocm_smi64) virtualisation — the rocm-smi twin of hooks_smi.cpp
// (reference: nvmlDeviceGetCount_v2, handle_remap and nvmlDeviceGetMemoryInfo,
// SURVEY.md §2.6 E1c).
//
// rsmi names devices by index, and its indices enumerate every GPU of the node
// (sysfs is not namespaced).  When the container's PCI addresses are known
// (hooks_smi.cpp container_bdfs), rsmi_num_monitor_devices reports the
// container's GPU count and an application's index i is the container's
// ordinal i: each hooked per-device entry point below translates it to the
// physical rsmi index whose PCI address is ordinal i's (rsmi_dev_pci_id_get),
// and refuses an index past the container's devices.  Calls that libamd_smi
// makes into its bundled rocm-smi keep physical indices.  Without known
// addresses, indices pass through and equal the container ordinals.
#include <rocm_smi/rocm_smi.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

#include "common.h"
#include "real.h"
#include "state.h"

using namespace vgpu;

namespace vgpu {
const std::vector<std::string>& container_bdfs();
int ordinal_of_bdf(const std::string& bdf);
}  // namespace vgpu

#define REAL_RSMI(name) \
  ((decltype(&::name))smi_real(#name, __builtin_return_address(0), rsmi_lib_handle))

namespace {

std::mutex g_mu;
bool g_ready = false;
std::vector<uint32_t> g_phys;  // container ordinal -> physical rsmi index (empty: no remap)

void map_locked() {
  if (g_ready) return;
  g_ready = true;
  ensure_init();
  if (!st().enabled || container_bdfs().empty()) return;
  auto num = (rsmi_status_t(*)(uint32_t*))smi_real("rsmi_num_monitor_devices", nullptr, rsmi_lib_handle);
  auto pci = (rsmi_status_t(*)(uint32_t, uint64_t*))smi_real("rsmi_dev_pci_id_get", nullptr, rsmi_lib_handle);
  uint32_t n = 0;
  if (!num || !pci || num(&n) != RSMI_STATUS_SUCCESS) return;
  std::vector<uint32_t> phys(container_bdfs().size(), UINT32_MAX);
  for (uint32_t p = 0; p < n; ++p) {
    uint64_t id = 0;
    if (pci(p, &id) != RSMI_STATUS_SUCCESS) continue;
    // BDFID = (domain << 32) | (bus << 8) | (device << 3) | function
    char b[32];
    snprintf(b, sizeof b, "%04x:%02x:%02x.%x", (unsigned)((id >> 32) & 0xffffffffu), (unsigned)((id >> 8) & 0xff),
             (unsigned)((id >> 3) & 0x1f), (unsigned)(id & 0x7));
    const int ord = ordinal_of_bdf(b);
    if (ord >= 0 && ord < (int)phys.size()) phys[ord] = p;
  }
  // Every ordinal found: remap.  A container whose GPUs rsmi does not list
  // (partial view) keeps the pass-through rule rather than half a mapping.
  if (std::find(phys.begin(), phys.end(), UINT32_MAX) == phys.end()) g_phys = phys;
}

// The physical index for an application's index `dv` (false: not one of the
// container's devices).  Calls from inside an smi library pass through.
bool remap(uint32_t dv, void* ret, uint32_t* out) {
  *out = dv;
  if (called_from_smi_lib(ret)) return true;
  std::lock_guard<std::mutex> g(g_mu);
  map_locked();
  if (g_phys.empty()) return true;
  if (dv >= g_phys.size()) return false;
  *out = g_phys[dv];
  return true;
}

bool rsmi_vram(rsmi_memory_type_t t) {
  return t == RSMI_MEM_TYPE_VRAM || t == RSMI_MEM_TYPE_VIS_VRAM;
}

uint64_t rsmi_limit(uint32_t ordinal) {
  ensure_init();
  if (!st().enabled || ordinal >= VGPU_MAX_DEVICES) return 0;
  return mem_limit((int)ordinal);
}

}  // namespace

// A per-device rsmi entry point whose device index is remapped: name, then the
// parameters and the arguments after dv_ind, each list in parentheses.
#define VGPU_EXPAND(...) __VA_ARGS__
#define VGPU_RSMI_REMAP(name, PARAMS, ARGS)                                                    \
  __attribute__((visibility("default"))) rsmi_status_t name(uint32_t dv_ind, VGPU_EXPAND PARAMS) { \
    auto real = REAL_RSMI(name);                                                               \
    uint32_t p;                                                                                \
    if (!remap(dv_ind, __builtin_return_address(0), &p)) return RSMI_STATUS_INVALID_ARGS;      \
    return real(p, VGPU_EXPAND ARGS);                                                          \
  }

extern "C" {

__attribute__((visibility("default"))) rsmi_status_t rsmi_num_monitor_devices(uint32_t* n) {
  rsmi_status_t rc = REAL_RSMI(rsmi_num_monitor_devices)(n);
  if (rc != RSMI_STATUS_SUCCESS || !n || called_from_smi_lib(__builtin_return_address(0))) return rc;
  std::lock_guard<std::mutex> g(g_mu);
  map_locked();
  if (!g_phys.empty()) *n = (uint32_t)g_phys.size();
  return rc;
}

__attribute__((visibility("default"))) rsmi_status_t rsmi_dev_memory_total_get(
    uint32_t dv_ind, rsmi_memory_type_t type, uint64_t* total) {
  void* ret = __builtin_return_address(0);
  uint32_t p;
  if (!remap(dv_ind, ret, &p)) return RSMI_STATUS_INVALID_ARGS;
  rsmi_status_t rc = REAL_RSMI(rsmi_dev_memory_total_get)(p, type, total);
  if (rc != RSMI_STATUS_SUCCESS || !total || !rsmi_vram(type) || called_from_smi_lib(ret)) return rc;
  if (uint64_t lim = rsmi_limit(dv_ind)) *total = lim;
  return rc;
}

__attribute__((visibility("default"))) rsmi_status_t rsmi_dev_memory_usage_get(
    uint32_t dv_ind, rsmi_memory_type_t type, uint64_t* used) {
  void* ret = __builtin_return_address(0);
  uint32_t p;
  if (!remap(dv_ind, ret, &p)) return RSMI_STATUS_INVALID_ARGS;
  rsmi_status_t rc = REAL_RSMI(rsmi_dev_memory_usage_get)(p, type, used);
  if (rc != RSMI_STATUS_SUCCESS || !used || !rsmi_vram(type) || called_from_smi_lib(ret)) return rc;
  if (uint64_t lim = rsmi_limit(dv_ind)) {
    State& s = st();
    uint64_t u = s.region ? region_device_used(s.region, (int)dv_ind) : 0;
    *used = std::min<uint64_t>(u, lim);
  }
  return rc;
}

VGPU_RSMI_REMAP(rsmi_dev_pci_id_get, (uint64_t* bdfid), (bdfid))
VGPU_RSMI_REMAP(rsmi_dev_id_get, (uint16_t* id), (id))
VGPU_RSMI_REMAP(rsmi_dev_vendor_id_get, (uint16_t* id), (id))
VGPU_RSMI_REMAP(rsmi_dev_name_get, (char* name, size_t len), (name, len))
VGPU_RSMI_REMAP(rsmi_dev_brand_get, (char* brand, uint32_t len), (brand, len))
VGPU_RSMI_REMAP(rsmi_dev_serial_number_get, (char* serial, uint32_t len), (serial, len))
VGPU_RSMI_REMAP(rsmi_dev_unique_id_get, (uint64_t* id), (id))
VGPU_RSMI_REMAP(rsmi_dev_guid_get, (uint64_t* guid), (guid))
VGPU_RSMI_REMAP(rsmi_dev_node_id_get, (uint32_t* node), (node))
VGPU_RSMI_REMAP(rsmi_dev_busy_percent_get, (uint32_t* pct), (pct))
VGPU_RSMI_REMAP(rsmi_dev_memory_busy_percent_get, (uint32_t* pct), (pct))
VGPU_RSMI_REMAP(rsmi_dev_temp_metric_get, (uint32_t sensor, rsmi_temperature_metric_t metric, int64_t* t),
                (sensor, metric, t))
VGPU_RSMI_REMAP(rsmi_dev_power_get, (uint64_t* power, RSMI_POWER_TYPE* type), (power, type))
VGPU_RSMI_REMAP(rsmi_dev_gpu_metrics_info_get, (rsmi_gpu_metrics_t* m), (m))
VGPU_RSMI_REMAP(rsmi_dev_ecc_count_get, (rsmi_gpu_block_t block, rsmi_error_count_t* ec), (block, ec))
VGPU_RSMI_REMAP(rsmi_dev_gpu_clk_freq_get, (rsmi_clk_type_t clk, rsmi_frequencies_t* f), (clk, f))

// Compute processes on the node (KFD), filtered to this container's own.
__attribute__((visibility("default"))) rsmi_status_t rsmi_compute_process_info_get(
    rsmi_process_info_t* procs, uint32_t* num_items) {
  auto real = REAL_RSMI(rsmi_compute_process_info_get);
  ensure_init();
  if (!st().enabled || !num_items) return real(procs, num_items);
  uint32_t n = 0;
  rsmi_status_t rc = real(nullptr, &n);
  if (rc != RSMI_STATUS_SUCCESS && rc != RSMI_STATUS_INSUFFICIENT_SIZE) return rc;
  std::vector<rsmi_process_info_t> all(n + 16);
  uint32_t got = (uint32_t)all.size();
  rc = real(all.data(), &got);
  if (rc != RSMI_STATUS_SUCCESS && rc != RSMI_STATUS_INSUFFICIENT_SIZE) return rc;
  const std::vector<int> mine = container_host_pids();
  const uint32_t cap = procs ? *num_items : 0;
  uint32_t k = 0;
  for (uint32_t i = 0; i < got && i < all.size(); ++i) {
    if (std::find(mine.begin(), mine.end(), (int)all[i].process_id) == mine.end()) continue;
    if (k < cap) procs[k] = all[i];
    ++k;
  }
  *num_items = k;
  return procs && k > cap ? RSMI_STATUS_INSUFFICIENT_SIZE : RSMI_STATUS_SUCCESS;
}

}  // extern "C"
