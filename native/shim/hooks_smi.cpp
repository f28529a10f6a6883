// amdsmi / rocm-smi virtualisation: inside a vGPU container, `amd-smi`,
// `rocm-smi`, and PyTorch's amdsmi queries see the container's GPUs only, in
// the container's (HIP) order, with the container's HBM cap as their VRAM, the
// container's usage as "used" and the container's processes as theirs.
//
// Reference behaviour: libvgpu.so hooks 247 nvml* entry points; the ones with
// behaviour are nvmlDeviceGetMemoryInfo (1190 B) / _v2 (1214 B), which report
// the container's limit and usage, the handle <-> index remap `handle_remap`
// (640 B) with nvmlDeviceGetCount_v2 (186 B) / nvmlDeviceGetHandleByIndex_v2
// (238 B), and the process lists; everything else passes through (SURVEY.md
// §2.6 E1c).  The MI355X equivalents are amdsmi_get_processor_handles /
// amdsmi_get_socket_handles (device list), amdsmi_get_gpu_memory_total /
// _usage, amdsmi_get_gpu_vram_usage / _info, amdsmi_get_gpu_process_list
// (libamd_smi) and their rocm-smi twins (hooks_rsmi.cpp).  Lookups made by
// ctypes through a dlopen handle reach these via the dlsym interposer
// (dlsym.cpp).
//
// Device identity.  sysfs is not namespaced: an smi library in
// a pod that holds physical GPU 5 enumerates all eight GPUs of the node, and
// enumeration order says nothing about which one is the container's ordinal 0.
// The device plugin passes each ordinal's PCI address (VGPU_DEVICE_BDF_<i>,
// vgpu/deviceplugin/allocate.py); without it, the HIP runtime's answer
// (hipDeviceGetPCIBusId) when the process has already loaded HIP.  A GPU handle
// whose BDF is none of the container's is not listed; ours are listed in
// ordinal order, and every memory query is indexed by the ordinal the BDF
// names.  With no BDF known (a container started outside the device plugin,
// before HIP) the old rule applies: enumeration order = ordinal, no filtering.
//
// Process lists are filtered to this container's processes: the host pids of
// its region's slots as resolved by hostpid.cpp.  A process whose host pid is
// unknown is hidden rather than guessed.
#include <amd_smi/amdsmi.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.h"
#include "real.h"
#include "state.h"

using namespace vgpu;

namespace vgpu {

// PCI address of every container ordinal ("dddd:bb:dd.f", lower case), from
// the device plugin's env or the loaded HIP runtime; empty when unknown.
const std::vector<std::string>& container_bdfs() {
  static std::once_flag once;
  static std::vector<std::string> out;
  std::call_once(once, [] {
    auto norm = [](const char* v) -> std::string {
      unsigned dom = 0, bus = 0, dev = 0, fn = 0;
      if (sscanf(v, "%x:%x:%x.%x", &dom, &bus, &dev, &fn) != 4) return {};
      char b[32];
      snprintf(b, sizeof b, "%04x:%02x:%02x.%x", dom, bus, dev, fn);
      return b;
    };
    for (int i = 0; i < VGPU_MAX_DEVICES; ++i) {
      char name[40];
      snprintf(name, sizeof name, "VGPU_DEVICE_BDF_%d", i);
      const char* v = getenv(name);
      if (!v || !*v) break;
      const std::string b = norm(v);
      if (b.empty()) break;
      out.push_back(b);
    }
    if (!out.empty()) return;
    // The HIP runtime, only if this process already loaded it (an smi-only
    // tool must not start a HIP runtime).
    static const char* names[] = {"libamdhip64.so.7", "libamdhip64.so"};
    void* h = nullptr;
    for (const char* n : names)
      if ((h = dlopen(n, RTLD_NOLOAD | RTLD_LAZY))) break;
    if (!h) return;
    auto count = (hipError_t(*)(int*))real_dlsym(h, "hipGetDeviceCount");
    auto bus = (hipError_t(*)(char*, int, int))real_dlsym(h, "hipDeviceGetPCIBusId");
    int n = 0;
    if (!count || !bus || count(&n) != hipSuccess) return;
    for (int i = 0; i < n && i < VGPU_MAX_DEVICES; ++i) {
      char b[64] = {};
      if (bus(b, sizeof b, i) != hipSuccess) {
        out.clear();
        return;
      }
      const std::string s = norm(b);
      if (s.empty()) {
        out.clear();
        return;
      }
      out.push_back(s);
    }
  });
  return out;
}

// Container ordinal of a PCI address, -1 when it is not one of ours, -2 when
// the container's addresses are unknown.
int ordinal_of_bdf(const std::string& bdf) {
  const auto& mine = container_bdfs();
  if (mine.empty()) return -2;
  auto it = std::find(mine.begin(), mine.end(), bdf);
  return it == mine.end() ? -1 : (int)(it - mine.begin());
}

}  // namespace vgpu

namespace {

#define REAL_SMI(name) \
  ((decltype(&::name))smi_real(#name, __builtin_return_address(0), amdsmi_lib_handle))

std::mutex g_mu;
bool g_ready = false;
bool g_by_bdf = false;                                     // identity by PCI address
std::vector<amdsmi_processor_handle> g_gpus;               // every GPU handle, enumeration order
std::unordered_map<amdsmi_processor_handle, int> g_ord;    // handle -> container ordinal (-1: not ours)

std::string bdf_string(amdsmi_bdf_t b) {
  char s[32];
  snprintf(s, sizeof s, "%04llx:%02x:%02x.%x", (unsigned long long)b.domain_number, (unsigned)b.bus_number,
           (unsigned)b.device_number, (unsigned)b.function_number);
  return s;
}

// Enumerate the GPU handles once (real calls) and map them to ordinals.
void enumerate_locked() {
  if (g_ready) return;
  auto socks_fn = (amdsmi_status_t(*)(uint32_t*, amdsmi_socket_handle*))smi_real(
      "amdsmi_get_socket_handles", nullptr, amdsmi_lib_handle);
  auto procs_fn = (amdsmi_status_t(*)(amdsmi_socket_handle, uint32_t*, amdsmi_processor_handle*))smi_real(
      "amdsmi_get_processor_handles", nullptr, amdsmi_lib_handle);
  auto type_fn = (amdsmi_status_t(*)(amdsmi_processor_handle, processor_type_t*))smi_real(
      "amdsmi_get_processor_type", nullptr, amdsmi_lib_handle);
  auto bdf_fn = (amdsmi_status_t(*)(amdsmi_processor_handle, amdsmi_bdf_t*))smi_real(
      "amdsmi_get_gpu_device_bdf", nullptr, amdsmi_lib_handle);
  if (!socks_fn || !procs_fn || !type_fn) return;
  uint32_t ns = 0;
  if (socks_fn(&ns, nullptr) != AMDSMI_STATUS_SUCCESS || !ns) return;
  std::vector<amdsmi_socket_handle> socks(ns);
  if (socks_fn(&ns, socks.data()) != AMDSMI_STATUS_SUCCESS) return;
  for (uint32_t s = 0; s < ns; ++s) {
    uint32_t np = 0;
    if (procs_fn(socks[s], &np, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
    std::vector<amdsmi_processor_handle> ps(np);
    if (procs_fn(socks[s], &np, ps.data()) != AMDSMI_STATUS_SUCCESS) continue;
    for (uint32_t i = 0; i < np; ++i) {
      processor_type_t t = AMDSMI_PROCESSOR_TYPE_UNKNOWN;
      if (type_fn(ps[i], &t) == AMDSMI_STATUS_SUCCESS && t == AMDSMI_PROCESSOR_TYPE_AMD_GPU) g_gpus.push_back(ps[i]);
    }
  }
  if (g_gpus.empty()) return;
  g_ready = true;
  ensure_init();
  g_by_bdf = st().enabled && bdf_fn && !container_bdfs().empty();
  for (size_t i = 0; i < g_gpus.size(); ++i) {
    int ord = (int)i;
    if (g_by_bdf) {
      amdsmi_bdf_t b{};
      ord = bdf_fn(g_gpus[i], &b) == AMDSMI_STATUS_SUCCESS ? ordinal_of_bdf(bdf_string(b)) : -1;
    }
    g_ord[g_gpus[i]] = ord;
  }
}

// Container ordinal of GPU handle `h`; -1 when it is not the container's (or unknown).
int gpu_index(amdsmi_processor_handle h) {
  std::lock_guard<std::mutex> g(g_mu);
  enumerate_locked();
  auto it = g_ord.find(h);
  return it == g_ord.end() ? -1 : it->second;
}

bool filtering() {
  std::lock_guard<std::mutex> g(g_mu);
  enumerate_locked();
  return g_by_bdf;
}

// Is `h` a GPU of the node that is not this container's (listed only when not filtering)?
bool foreign_gpu(amdsmi_processor_handle h) {
  std::lock_guard<std::mutex> g(g_mu);
  enumerate_locked();
  if (!g_by_bdf) return false;
  auto it = g_ord.find(h);
  return it != g_ord.end() && it->second < 0;
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

// The container's GPU handles of `all` (one socket's processors), ordinal order,
// the socket's other processors (CPUs, ...) after them.
std::vector<amdsmi_processor_handle> visible_of(const std::vector<amdsmi_processor_handle>& all) {
  std::vector<std::pair<int, amdsmi_processor_handle>> gpus;
  std::vector<amdsmi_processor_handle> other;
  {
    std::lock_guard<std::mutex> g(g_mu);
    for (auto h : all) {
      auto it = g_ord.find(h);
      if (it == g_ord.end())
        other.push_back(h);
      else if (it->second >= 0)
        gpus.push_back({it->second, h});
    }
  }
  std::sort(gpus.begin(), gpus.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  std::vector<amdsmi_processor_handle> out;
  for (auto& p : gpus) out.push_back(p.second);
  out.insert(out.end(), other.begin(), other.end());
  return out;
}

}  // namespace

extern "C" {

// Device list: only the container's GPUs, in its order (handle_remap /
// nvmlDeviceGetCount_v2 / nvmlDeviceGetHandleByIndex_v2 of the reference).
__attribute__((visibility("default"))) amdsmi_status_t amdsmi_get_processor_handles(
    amdsmi_socket_handle sock, uint32_t* count, amdsmi_processor_handle* handles) {
  auto real = REAL_SMI(amdsmi_get_processor_handles);
  if (!count || called_from_smi_lib(__builtin_return_address(0)) || !filtering()) return real(sock, count, handles);
  uint32_t n = 0;
  amdsmi_status_t rc = real(sock, &n, nullptr);
  if (rc != AMDSMI_STATUS_SUCCESS) return rc;
  std::vector<amdsmi_processor_handle> all(n);
  if (n && (rc = real(sock, &n, all.data())) != AMDSMI_STATUS_SUCCESS) return rc;
  all.resize(n);
  const auto vis = visible_of(all);
  if (handles)
    for (uint32_t i = 0; i < vis.size() && i < *count; ++i) handles[i] = vis[i];
  *count = (uint32_t)vis.size();
  return AMDSMI_STATUS_SUCCESS;
}

__attribute__((visibility("default"))) amdsmi_status_t amdsmi_get_processor_handles_by_type(
    amdsmi_socket_handle sock, processor_type_t type, amdsmi_processor_handle* handles, uint32_t* count) {
  auto real = REAL_SMI(amdsmi_get_processor_handles_by_type);
  if (!count || type != AMDSMI_PROCESSOR_TYPE_AMD_GPU || called_from_smi_lib(__builtin_return_address(0)) ||
      !filtering())
    return real(sock, type, handles, count);
  uint32_t n = 0;
  amdsmi_status_t rc = real(sock, type, nullptr, &n);
  if (rc != AMDSMI_STATUS_SUCCESS) return rc;
  std::vector<amdsmi_processor_handle> all(n);
  if (n && (rc = real(sock, type, all.data(), &n)) != AMDSMI_STATUS_SUCCESS) return rc;
  all.resize(n);
  const auto vis = visible_of(all);
  if (handles)
    for (uint32_t i = 0; i < vis.size() && i < *count; ++i) handles[i] = vis[i];
  *count = (uint32_t)vis.size();
  return AMDSMI_STATUS_SUCCESS;
}

// Sockets whose GPUs are all other containers' are not listed either.
__attribute__((visibility("default"))) amdsmi_status_t amdsmi_get_socket_handles(uint32_t* count,
                                                                                amdsmi_socket_handle* handles) {
  auto real = REAL_SMI(amdsmi_get_socket_handles);
  if (!count || called_from_smi_lib(__builtin_return_address(0)) || !filtering()) return real(count, handles);
  uint32_t n = 0;
  amdsmi_status_t rc = real(&n, nullptr);
  if (rc != AMDSMI_STATUS_SUCCESS) return rc;
  std::vector<amdsmi_socket_handle> all(n);
  if (n && (rc = real(&n, all.data())) != AMDSMI_STATUS_SUCCESS) return rc;
  auto procs_fn = (amdsmi_status_t(*)(amdsmi_socket_handle, uint32_t*, amdsmi_processor_handle*))smi_real(
      "amdsmi_get_processor_handles", nullptr, amdsmi_lib_handle);
  std::vector<amdsmi_socket_handle> keep;
  for (uint32_t s = 0; s < n; ++s) {
    uint32_t np = 0;
    std::vector<amdsmi_processor_handle> ps;
    if (procs_fn && procs_fn(all[s], &np, nullptr) == AMDSMI_STATUS_SUCCESS && np) {
      ps.resize(np);
      if (procs_fn(all[s], &np, ps.data()) != AMDSMI_STATUS_SUCCESS) np = 0;
      ps.resize(np);
    }
    if (ps.empty() || !visible_of(ps).empty()) keep.push_back(all[s]);
  }
  if (handles)
    for (uint32_t i = 0; i < keep.size() && i < *count; ++i) handles[i] = keep[i];
  *count = (uint32_t)keep.size();
  return AMDSMI_STATUS_SUCCESS;
}

// Another container's GPU by address: not found from inside this one.
__attribute__((visibility("default"))) amdsmi_status_t amdsmi_get_processor_handle_from_bdf(
    amdsmi_bdf_t bdf, amdsmi_processor_handle* h) {
  amdsmi_status_t rc = REAL_SMI(amdsmi_get_processor_handle_from_bdf)(bdf, h);
  if (rc == AMDSMI_STATUS_SUCCESS && h && !called_from_smi_lib(__builtin_return_address(0)) && foreign_gpu(*h)) {
    *h = nullptr;
    return AMDSMI_STATUS_NOT_FOUND;
  }
  return rc;
}

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
