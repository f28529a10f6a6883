// libvgpu_smi: device discovery and telemetry for the device plugin and the
// node monitor (see include/vgpu/smi.h).
//
// amdsmi backend: libamd_smi.so is dlopen'ed (never linked) so the same binary
// runs on hosts without ROCm and in tests against the fixture-driven fake.
// sysfs backend: KFD topology (/sys/class/kfd/kfd/topology/nodes/N) + PCI
// sysfs; VGPU_SYSFS_ROOT relocates "/" for tests.
#include "vgpu/smi.h"

#include <amd_smi/amdsmi.h>
#include <dirent.h>
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

namespace {

std::mutex g_mu;
std::string g_backend = "none";

// ---------------------------------------------------------------------- amdsmi
struct AmdSmi {
  void* h = nullptr;
#define F(name) decltype(&::name) name = nullptr
  F(amdsmi_init);
  F(amdsmi_shut_down);
  F(amdsmi_get_socket_handles);
  F(amdsmi_get_processor_handles);
  F(amdsmi_get_processor_type);
  F(amdsmi_get_gpu_device_uuid);
  F(amdsmi_get_gpu_device_bdf);
  F(amdsmi_get_gpu_asic_info);
  F(amdsmi_get_gpu_memory_total);
  F(amdsmi_get_gpu_memory_usage);
  F(amdsmi_get_gpu_topo_numa_affinity);
  F(amdsmi_topo_get_link_type);
  F(amdsmi_get_gpu_compute_partition);
  F(amdsmi_get_gpu_memory_partition);
  F(amdsmi_get_gpu_activity);
  F(amdsmi_get_gpu_process_list);
  F(amdsmi_get_gpu_kfd_info);
  F(amdsmi_get_gpu_enumeration_info);
  F(amdsmi_get_xgmi_info);
  F(amdsmi_init_gpu_event_notification);
  F(amdsmi_set_gpu_event_notification_mask);
  F(amdsmi_get_gpu_event_notification);
  F(amdsmi_get_gpu_total_ecc_count);
  F(amdsmi_get_power_info);
  F(amdsmi_get_temp_metric);
  F(amdsmi_get_gpu_metrics_info);
#undef F
  std::vector<amdsmi_processor_handle> gpus;
  bool events_on = false;

  bool load() {
    const char* env = getenv("VGPU_AMDSMI_LIB");
    const char* cands[] = {env, "libamd_smi.so", "/opt/rocm/lib/libamd_smi.so", nullptr};
    for (const char* c : cands) {
      if (!c) continue;
      h = dlopen(c, RTLD_NOW | RTLD_LOCAL);
      if (h) break;
    }
    if (!h) return false;
#define L(name) name = (decltype(name))dlsym(h, #name)
    L(amdsmi_init); L(amdsmi_shut_down); L(amdsmi_get_socket_handles);
    L(amdsmi_get_processor_handles); L(amdsmi_get_processor_type);
    L(amdsmi_get_gpu_device_uuid); L(amdsmi_get_gpu_device_bdf); L(amdsmi_get_gpu_asic_info);
    L(amdsmi_get_gpu_memory_total); L(amdsmi_get_gpu_memory_usage);
    L(amdsmi_get_gpu_topo_numa_affinity); L(amdsmi_topo_get_link_type);
    L(amdsmi_get_gpu_compute_partition); L(amdsmi_get_gpu_memory_partition);
    L(amdsmi_get_gpu_activity); L(amdsmi_get_gpu_process_list); L(amdsmi_get_gpu_kfd_info);
    L(amdsmi_get_gpu_enumeration_info); L(amdsmi_get_xgmi_info);
    L(amdsmi_init_gpu_event_notification); L(amdsmi_set_gpu_event_notification_mask);
    L(amdsmi_get_gpu_event_notification);
    L(amdsmi_get_gpu_total_ecc_count); L(amdsmi_get_power_info); L(amdsmi_get_temp_metric);
    L(amdsmi_get_gpu_metrics_info);
#undef L
    if (!amdsmi_init || !amdsmi_get_socket_handles || !amdsmi_get_processor_handles) return false;
    if (amdsmi_init(AMDSMI_INIT_AMD_GPUS) != AMDSMI_STATUS_SUCCESS) return false;
    uint32_t ns = 0;
    if (amdsmi_get_socket_handles(&ns, nullptr) != AMDSMI_STATUS_SUCCESS) return false;
    std::vector<amdsmi_socket_handle> socks(ns);
    amdsmi_get_socket_handles(&ns, socks.data());
    for (auto s : socks) {
      uint32_t np = 0;
      if (amdsmi_get_processor_handles(s, &np, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
      std::vector<amdsmi_processor_handle> ps(np);
      amdsmi_get_processor_handles(s, &np, ps.data());
      for (auto p : ps) {
        processor_type_t t = AMDSMI_PROCESSOR_TYPE_UNKNOWN;
        if (amdsmi_get_processor_type && amdsmi_get_processor_type(p, &t) == AMDSMI_STATUS_SUCCESS &&
            t != AMDSMI_PROCESSOR_TYPE_AMD_GPU)
          continue;
        gpus.push_back(p);
      }
    }
    return true;
  }

  void telemetry(int i, vgpu_smi_telemetry_t* t) {
    amdsmi_processor_handle p = gpus[i];
    memset(t, 0, sizeof(*t));
    amdsmi_error_count_t ec;
    if (amdsmi_get_gpu_total_ecc_count && amdsmi_get_gpu_total_ecc_count(p, &ec) == AMDSMI_STATUS_SUCCESS) {
      t->ecc_correctable = ec.correctable_count;
      t->ecc_uncorrectable = ec.uncorrectable_count;
      t->ecc_deferred = ec.deferred_count;
      t->valid |= VGPU_TELEM_ECC;
    }
    amdsmi_power_info_t pw;
    if (amdsmi_get_power_info && amdsmi_get_power_info(p, &pw) == AMDSMI_STATUS_SUCCESS) {
      uint32_t w = pw.current_socket_power;
      if (w == 0 || w == 0xFFFFu || w == 0xFFFFFFFFu) w = pw.average_socket_power;
      if (w == 0xFFFFu || w == 0xFFFFFFFFu) w = 0;
      t->power_w = w;
      t->valid |= VGPU_TELEM_POWER;
    }
    if (amdsmi_get_temp_metric) {
      int64_t v = 0;
      bool any = false;
      if (amdsmi_get_temp_metric(p, AMDSMI_TEMPERATURE_TYPE_EDGE, AMDSMI_TEMP_CURRENT, &v) == AMDSMI_STATUS_SUCCESS) {
        t->temp_edge_c = (int32_t)v;
        any = true;
      }
      if (amdsmi_get_temp_metric(p, AMDSMI_TEMPERATURE_TYPE_HOTSPOT, AMDSMI_TEMP_CURRENT, &v) == AMDSMI_STATUS_SUCCESS) {
        t->temp_hotspot_c = (int32_t)v;
        any = true;
      }
      if (amdsmi_get_temp_metric(p, AMDSMI_TEMPERATURE_TYPE_VRAM, AMDSMI_TEMP_CURRENT, &v) == AMDSMI_STATUS_SUCCESS) {
        t->temp_mem_c = (int32_t)v;
        any = true;
      }
      if (any) t->valid |= VGPU_TELEM_TEMP;
    }
    if (amdsmi_get_gpu_metrics_info) {
      amdsmi_gpu_metrics_t* m = new amdsmi_gpu_metrics_t;
      if (amdsmi_get_gpu_metrics_info(p, m) == AMDSMI_STATUS_SUCCESS) {
        for (int l = 0; l < AMDSMI_MAX_NUM_XGMI_LINKS; ++l) {
          if (m->xgmi_read_data_acc[l] != UINT64_MAX) t->xgmi_read_kb += m->xgmi_read_data_acc[l];
          if (m->xgmi_write_data_acc[l] != UINT64_MAX) t->xgmi_write_kb += m->xgmi_write_data_acc[l];
        }
        t->valid |= VGPU_TELEM_XGMI;
      }
      delete m;
    }
  }

  void fill(int i, vgpu_smi_device_t* d) {
    amdsmi_processor_handle p = gpus[i];
    memset(d, 0, sizeof(*d));
    d->index = (uint32_t)i;
    d->health = 1;
    d->numa_node = -1;
    unsigned int len = VGPU_SMI_STR;
    if (amdsmi_get_gpu_device_uuid) amdsmi_get_gpu_device_uuid(p, &len, d->uuid);
    amdsmi_bdf_t bdf;
    if (amdsmi_get_gpu_device_bdf && amdsmi_get_gpu_device_bdf(p, &bdf) == AMDSMI_STATUS_SUCCESS)
      snprintf(d->bdf, sizeof d->bdf, "%04llx:%02x:%02x.%x", (unsigned long long)bdf.domain_number,
               (unsigned)bdf.bus_number, (unsigned)bdf.device_number, (unsigned)bdf.function_number);
    amdsmi_asic_info_t asic;
    if (amdsmi_get_gpu_asic_info && amdsmi_get_gpu_asic_info(p, &asic) == AMDSMI_STATUS_SUCCESS) {
      snprintf(d->name, sizeof d->name, "%s", asic.market_name);
      d->vendor_id = asic.vendor_id;
      d->device_id = asic.device_id;
      if (asic.num_of_compute_units != 0xFFFFFFFFu) d->cus = asic.num_of_compute_units;
    }
    if (amdsmi_get_gpu_memory_total)
      amdsmi_get_gpu_memory_total(p, AMDSMI_MEM_TYPE_VRAM, &d->vram_total);
    if (amdsmi_get_gpu_memory_usage)
      amdsmi_get_gpu_memory_usage(p, AMDSMI_MEM_TYPE_VRAM, &d->vram_used);
    int32_t numa = -1;
    if (amdsmi_get_gpu_topo_numa_affinity &&
        amdsmi_get_gpu_topo_numa_affinity(p, &numa) == AMDSMI_STATUS_SUCCESS)
      d->numa_node = numa;
    if (amdsmi_get_gpu_compute_partition)
      amdsmi_get_gpu_compute_partition(p, d->compute_partition, sizeof d->compute_partition);
    if (amdsmi_get_gpu_memory_partition)
      amdsmi_get_gpu_memory_partition(p, d->memory_partition, sizeof d->memory_partition);
    amdsmi_engine_usage_t act;
    if (amdsmi_get_gpu_activity && amdsmi_get_gpu_activity(p, &act) == AMDSMI_STATUS_SUCCESS) {
      d->gfx_activity = act.gfx_activity;
      d->umc_activity = act.umc_activity;
    }
    amdsmi_kfd_info_t kfd;
    if (amdsmi_get_gpu_kfd_info && amdsmi_get_gpu_kfd_info(p, &kfd) == AMDSMI_STATUS_SUCCESS &&
        kfd.kfd_id != 0xFFFFFFFFFFFFFFFFull) {
      d->kfd_gpu_id = (uint32_t)kfd.kfd_id;
      if (kfd.current_partition_id != 0xFFFFFFFFu) d->partition_id = kfd.current_partition_id;
    }
    amdsmi_enumeration_info_t en;
    if (amdsmi_get_gpu_enumeration_info &&
        amdsmi_get_gpu_enumeration_info(p, &en) == AMDSMI_STATUS_SUCCESS) {
      d->render_minor = en.drm_render;
      d->card = en.drm_card;
    }
    amdsmi_xgmi_info_t xg;
    if (amdsmi_get_xgmi_info && amdsmi_get_xgmi_info(p, &xg) == AMDSMI_STATUS_SUCCESS)
      d->xgmi_hive = xg.xgmi_hive_id;
  }
};

AmdSmi* g_smi = nullptr;

// ----------------------------------------------------------------------- sysfs
struct SysfsDev {
  vgpu_smi_device_t d;
  std::string node_dir;
  std::string pci_dir;
};

std::vector<SysfsDev> g_sysfs;

std::string root_path(const std::string& p) {
  const char* r = getenv("VGPU_SYSFS_ROOT");
  return r && *r ? std::string(r) + p : p;
}

bool read_file(const std::string& path, std::string& out) {
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return false;
  char buf[4096];
  size_t n = fread(buf, 1, sizeof buf - 1, f);
  fclose(f);
  buf[n] = 0;
  out = buf;
  while (!out.empty() && (out.back() == '\n' || out.back() == ' ')) out.pop_back();
  return true;
}

bool prop(const std::string& props, const char* key, uint64_t* v) {
  size_t klen = strlen(key);
  size_t pos = 0;
  while (pos < props.size()) {
    size_t eol = props.find('\n', pos);
    if (eol == std::string::npos) eol = props.size();
    if (props.compare(pos, klen, key) == 0 && pos + klen < props.size() && props[pos + klen] == ' ') {
      *v = strtoull(props.c_str() + pos + klen + 1, nullptr, 10);
      return true;
    }
    pos = eol + 1;
  }
  return false;
}

bool sysfs_load() {
  std::string base = root_path("/sys/class/kfd/kfd/topology/nodes");
  DIR* dir = opendir(base.c_str());
  if (!dir) return false;
  std::vector<int> ids;
  struct dirent* e;
  while ((e = readdir(dir)))
    if (isdigit((unsigned char)e->d_name[0])) ids.push_back(atoi(e->d_name));
  closedir(dir);
  std::sort(ids.begin(), ids.end());
  for (int id : ids) {
    std::string nd = base + "/" + std::to_string(id);
    std::string props, gpuid;
    if (!read_file(nd + "/properties", props)) continue;
    if (!read_file(nd + "/gpu_id", gpuid) || atoi(gpuid.c_str()) == 0) continue;  // CPU node
    SysfsDev s;
    memset(&s.d, 0, sizeof s.d);
    s.node_dir = nd;
    s.d.kfd_gpu_id = (uint32_t)strtoul(gpuid.c_str(), nullptr, 10);
    s.d.index = (uint32_t)g_sysfs.size();
    s.d.health = 1;
    uint64_t v = 0, simd = 0, simd_per_cu = 0;
    prop(props, "simd_count", &simd);
    prop(props, "simd_per_cu", &simd_per_cu);
    if (simd && simd_per_cu) s.d.cus = (uint32_t)(simd / simd_per_cu);
    if (prop(props, "num_xcc", &v)) s.d.num_xcc = (uint32_t)v;
    if (prop(props, "vendor_id", &v)) s.d.vendor_id = (uint32_t)v;
    if (prop(props, "device_id", &v)) s.d.device_id = v;
    if (prop(props, "drm_render_minor", &v)) s.d.render_minor = (uint32_t)v;
    if (prop(props, "hive_id", &v)) s.d.xgmi_hive = v;
    uint64_t uid = 0;
    if (prop(props, "unique_id", &uid) && uid)
      snprintf(s.d.uuid, sizeof s.d.uuid, "GPU-%016llx", (unsigned long long)uid);
    else
      snprintf(s.d.uuid, sizeof s.d.uuid, "GPU-kfd-%u", s.d.kfd_gpu_id);
    uint64_t loc = 0, dom = 0;
    prop(props, "location_id", &loc);
    prop(props, "domain", &dom);
    snprintf(s.d.bdf, sizeof s.d.bdf, "%04llx:%02llx:%02llx.%llx", (unsigned long long)dom,
             (unsigned long long)((loc >> 8) & 0xff), (unsigned long long)((loc >> 3) & 0x1f),
             (unsigned long long)(loc & 0x7));
    // VRAM: sum of the node's HBM memory banks
    std::string mb = nd + "/mem_banks";
    DIR* md = opendir(mb.c_str());
    if (md) {
      while ((e = readdir(md))) {
        if (!isdigit((unsigned char)e->d_name[0])) continue;
        std::string mp;
        uint64_t sz = 0, heap = 0;
        if (read_file(mb + "/" + e->d_name + "/properties", mp) && prop(mp, "size_in_bytes", &sz)) {
          prop(mp, "heap_type", &heap);
          if (heap == 1 || heap == 2 || heap == 0) s.d.vram_total += sz;  // FB public/private
        }
      }
      closedir(md);
    }
    s.pci_dir = root_path("/sys/bus/pci/devices/") + s.d.bdf;
    std::string t;
    s.d.numa_node = read_file(s.pci_dir + "/numa_node", t) ? atoi(t.c_str()) : -1;
    if (read_file(s.pci_dir + "/current_compute_partition", t))
      snprintf(s.d.compute_partition, sizeof s.d.compute_partition, "%s", t.c_str());
    if (read_file(s.pci_dir + "/current_memory_partition", t))
      snprintf(s.d.memory_partition, sizeof s.d.memory_partition, "%s", t.c_str());
    if (read_file(s.pci_dir + "/product_name", t) && !t.empty())
      snprintf(s.d.name, sizeof s.d.name, "%s", t.c_str());
    else
      snprintf(s.d.name, sizeof s.d.name, "AMD Instinct (device 0x%llx)", (unsigned long long)s.d.device_id);
    g_sysfs.push_back(s);
  }
  return !g_sysfs.empty();
}

void sysfs_refresh(SysfsDev& s) {
  std::string t;
  if (read_file(s.pci_dir + "/mem_info_vram_used", t)) s.d.vram_used = strtoull(t.c_str(), nullptr, 10);
  if (read_file(s.pci_dir + "/gpu_busy_percent", t)) s.d.gfx_activity = (uint32_t)atoi(t.c_str());
  if (read_file(s.pci_dir + "/mem_busy_percent", t)) s.d.umc_activity = (uint32_t)atoi(t.c_str());
}

}  // namespace

extern "C" {

__attribute__((visibility("default"))) int vgpu_smi_open(const char* backend) {
  std::lock_guard<std::mutex> g(g_mu);
  std::string b = backend && *backend ? backend : "auto";
  if (b == "auto" || b == "amdsmi") {
    auto* s = new AmdSmi();
    if (s->load() && !s->gpus.empty()) {
      g_smi = s;
      g_backend = "amdsmi";
      return (int)s->gpus.size();
    }
    delete s;
    if (b == "amdsmi") return -1;
  }
  g_sysfs.clear();
  if (sysfs_load()) {
    g_backend = "sysfs";
    return (int)g_sysfs.size();
  }
  g_backend = "none";
  return b == "sysfs" ? -1 : 0;
}

__attribute__((visibility("default"))) const char* vgpu_smi_backend(void) { return g_backend.c_str(); }

__attribute__((visibility("default"))) int vgpu_smi_count(void) {
  std::lock_guard<std::mutex> g(g_mu);
  if (g_smi) return (int)g_smi->gpus.size();
  return (int)g_sysfs.size();
}

__attribute__((visibility("default"))) int vgpu_smi_get(int i, vgpu_smi_device_t* out) {
  std::lock_guard<std::mutex> g(g_mu);
  if (g_smi) {
    if (i < 0 || i >= (int)g_smi->gpus.size()) return -1;
    g_smi->fill(i, out);
    return 0;
  }
  if (i < 0 || i >= (int)g_sysfs.size()) return -1;
  sysfs_refresh(g_sysfs[i]);
  *out = g_sysfs[i].d;
  return 0;
}

__attribute__((visibility("default"))) int vgpu_smi_link(int a, int b, uint64_t* hops, int32_t* type) {
  std::lock_guard<std::mutex> g(g_mu);
  *hops = 0;
  *type = VGPU_LINK_UNKNOWN;
  if (g_smi && g_smi->amdsmi_topo_get_link_type) {
    if (a < 0 || b < 0 || a >= (int)g_smi->gpus.size() || b >= (int)g_smi->gpus.size()) return -1;
    amdsmi_link_type_t t;
    if (g_smi->amdsmi_topo_get_link_type(g_smi->gpus[a], g_smi->gpus[b], hops, &t) != AMDSMI_STATUS_SUCCESS)
      return -1;
    *type = t == AMDSMI_LINK_TYPE_XGMI ? VGPU_LINK_XGMI : (t == AMDSMI_LINK_TYPE_PCIE ? VGPU_LINK_PCIE : 0);
    return 0;
  }
  if (a < 0 || b < 0 || a >= (int)g_sysfs.size() || b >= (int)g_sysfs.size()) return -1;
  // KFD io_links: type 11 = xGMI, 2 = PCIe
  std::string base = g_sysfs[a].node_dir + "/io_links";
  DIR* d = opendir(base.c_str());
  if (!d) return 0;
  struct dirent* e;
  std::string target = g_sysfs[b].node_dir.substr(g_sysfs[b].node_dir.rfind('/') + 1);
  while ((e = readdir(d))) {
    if (!isdigit((unsigned char)e->d_name[0])) continue;
    std::string p;
    if (!read_file(base + "/" + e->d_name + "/properties", p)) continue;
    uint64_t to = 0, t = 0, w = 0;
    prop(p, "node_to", &to);
    prop(p, "type", &t);
    prop(p, "weight", &w);
    if (std::to_string(to) == target) {
      *type = t == 11 ? VGPU_LINK_XGMI : (t == 2 ? VGPU_LINK_PCIE : VGPU_LINK_UNKNOWN);
      *hops = 1;
      break;
    }
  }
  closedir(d);
  return 0;
}

__attribute__((visibility("default"))) int vgpu_smi_processes(int i, vgpu_smi_proc_t* out, int max) {
  std::lock_guard<std::mutex> g(g_mu);
  if (g_smi && g_smi->amdsmi_get_gpu_process_list) {
    if (i < 0 || i >= (int)g_smi->gpus.size()) return -1;
    uint32_t n = 256;
    std::vector<amdsmi_proc_info_t> list(n);
    if (g_smi->amdsmi_get_gpu_process_list(g_smi->gpus[i], &n, list.data()) != AMDSMI_STATUS_SUCCESS)
      return -1;
    int k = 0;
    for (uint32_t j = 0; j < n && k < max; ++j, ++k) {
      out[k].pid = list[j].pid;
      out[k].cu_occupancy = list[j].cu_occupancy;
      out[k].vram_bytes = list[j].memory_usage.vram_mem;
      out[k].gfx_ns = list[j].engine_usage.gfx;
    }
    return k;
  }
  // sysfs: /sys/class/kfd/kfd/proc/<pid>/{vram_<gpuid>, stats_<gpuid>/cu_occupancy}
  if (i < 0 || i >= (int)g_sysfs.size()) return -1;
  std::string base = root_path("/sys/class/kfd/kfd/proc");
  DIR* d = opendir(base.c_str());
  if (!d) return 0;
  int k = 0;
  struct dirent* e;
  std::string gid = std::to_string(g_sysfs[i].d.kfd_gpu_id);
  while ((e = readdir(d)) && k < max) {
    if (!isdigit((unsigned char)e->d_name[0])) continue;
    std::string p = base + "/" + e->d_name, t;
    if (!read_file(p + "/vram_" + gid, t)) continue;
    out[k].pid = (uint32_t)atoi(e->d_name);
    out[k].vram_bytes = strtoull(t.c_str(), nullptr, 10);
    out[k].cu_occupancy = read_file(p + "/stats_" + gid + "/cu_occupancy", t) ? (uint32_t)atoi(t.c_str()) : 0;
    out[k].gfx_ns = 0;
    ++k;
  }
  closedir(d);
  return k;
}

namespace {

// sysfs telemetry: RAS error counters ("ue: N" / "ce: N" per block in
// <pci>/ras/*_err_count) and the first hwmon's power / temperature.
void sysfs_telemetry(const SysfsDev& s, vgpu_smi_telemetry_t* t) {
  std::string ras = s.pci_dir + "/ras";
  if (DIR* d = opendir(ras.c_str())) {
    while (struct dirent* e = readdir(d)) {
      std::string n = e->d_name;
      if (n.size() < 10 || n.compare(n.size() - 10, 10, "_err_count") != 0) continue;
      std::string body;
      if (!read_file(ras + "/" + n, body)) continue;
      unsigned long long ue = 0, ce = 0;
      const char* u = strstr(body.c_str(), "ue:");
      const char* c = strstr(body.c_str(), "ce:");
      if (u) ue = strtoull(u + 3, nullptr, 10);
      if (c) ce = strtoull(c + 3, nullptr, 10);
      t->ecc_uncorrectable += ue;
      t->ecc_correctable += ce;
      t->valid |= VGPU_TELEM_ECC;
    }
    closedir(d);
  }
  std::string hw = s.pci_dir + "/hwmon";
  if (DIR* d = opendir(hw.c_str())) {
    while (struct dirent* e = readdir(d)) {
      if (strncmp(e->d_name, "hwmon", 5)) continue;
      std::string base = hw + "/" + e->d_name, v;
      if (read_file(base + "/power1_average", v) || read_file(base + "/power1_input", v)) {
        t->power_w = (uint32_t)(strtoull(v.c_str(), nullptr, 10) / 1000000ull);  // microwatts
        t->valid |= VGPU_TELEM_POWER;
      }
      if (read_file(base + "/temp1_input", v)) {
        t->temp_edge_c = (int32_t)(atoll(v.c_str()) / 1000);  // millidegrees
        t->valid |= VGPU_TELEM_TEMP;
      }
      if (read_file(base + "/temp2_input", v)) t->temp_hotspot_c = (int32_t)(atoll(v.c_str()) / 1000);
      if (read_file(base + "/temp3_input", v)) t->temp_mem_c = (int32_t)(atoll(v.c_str()) / 1000);
      break;
    }
    closedir(d);
  }
}

}  // namespace

__attribute__((visibility("default"))) int vgpu_smi_telemetry(int i, vgpu_smi_telemetry_t* out) {
  std::lock_guard<std::mutex> g(g_mu);
  memset(out, 0, sizeof(*out));
  if (g_smi) {
    if (i < 0 || i >= (int)g_smi->gpus.size()) return -1;
    g_smi->telemetry(i, out);
    return 0;
  }
  if (i < 0 || i >= (int)g_sysfs.size()) return -1;
  sysfs_telemetry(g_sysfs[i], out);
  return 0;
}

__attribute__((visibility("default"))) int vgpu_smi_events(vgpu_smi_event_t* out, int max, int timeout_ms) {
  AmdSmi* s = g_smi;
  if (!s || !s->amdsmi_get_gpu_event_notification || !s->amdsmi_init_gpu_event_notification) {
    usleep((useconds_t)timeout_ms * 1000);
    return 0;
  }
  if (!s->events_on) {
    std::lock_guard<std::mutex> g(g_mu);
    uint64_t mask = AMDSMI_EVENT_MASK_FROM_INDEX(AMDSMI_EVT_NOTIF_VMFAULT) |
                    AMDSMI_EVENT_MASK_FROM_INDEX(AMDSMI_EVT_NOTIF_THERMAL_THROTTLE) |
                    AMDSMI_EVENT_MASK_FROM_INDEX(AMDSMI_EVT_NOTIF_GPU_PRE_RESET) |
                    AMDSMI_EVENT_MASK_FROM_INDEX(AMDSMI_EVT_NOTIF_GPU_POST_RESET);
    for (auto p : s->gpus) {
      s->amdsmi_init_gpu_event_notification(p);
      if (s->amdsmi_set_gpu_event_notification_mask) s->amdsmi_set_gpu_event_notification_mask(p, mask);
    }
    s->events_on = true;
  }
  uint32_t n = (uint32_t)std::min(max, 64);
  amdsmi_evt_notification_data_t data[64];
  if (s->amdsmi_get_gpu_event_notification(timeout_ms, &n, data) != AMDSMI_STATUS_SUCCESS) return 0;
  int k = 0;
  for (uint32_t j = 0; j < n; ++j) {
    int dev = -1;
    for (size_t q = 0; q < s->gpus.size(); ++q)
      if (s->gpus[q] == data[j].processor_handle) dev = (int)q;
    out[k].device = dev;
    out[k].type = (int32_t)data[j].event;
    snprintf(out[k].message, sizeof out[k].message, "%s", data[j].message);
    ++k;
  }
  return k;
}

__attribute__((visibility("default"))) void vgpu_smi_close(void) {
  std::lock_guard<std::mutex> g(g_mu);
  if (g_smi) {
    if (g_smi->amdsmi_shut_down) g_smi->amdsmi_shut_down();
    delete g_smi;
    g_smi = nullptr;
  }
  g_sysfs.clear();
  g_backend = "none";
}

}  // extern "C"
