// Fixture-driven fake of libamd_smi.so (the subset libvgpu_smi uses), the
// MI355X equivalent of the reference's fake libcndev.so
// (pkg/device-plugin/mlu/cndev/mock/cndev.c:22-39: every call answers from the
// JSON file named by $MOCK_JSON).  Fixture path: $VGPU_FAKE_AMDSMI_JSON.
//
// {"gpus":[{"uuid":..,"bdf":"0000:05:00.0","name":..,"vram":N,"vram_used":N,"cus":256,
//           "numa":0,"render":128,"card":0,"kfd_id":N,"hive":N,"partition":"SPX",
//           "mem_partition":"NPS1","partition_id":0,"gfx":0,"umc":0,"vendor":4098,
//           "processes":[{"pid":1,"vram":N,"cu":N,"gfx_ns":N}]}],
//  "link":"xgmi"|"pcie", "events":[{"gpu":0,"type":3,"message":".."}]}
// Telemetry ($VGPU_FAKE_AMDSMI_TELEMETRY, re-read on every call so a test can
// inject ECC errors while the plugin runs):
// {"0": {"ecc_ue":N,"ecc_ce":N,"power":W,"temp_edge":C,"temp_hotspot":C,"temp_mem":C,
//        "xgmi_read_kb":N,"xgmi_write_kb":N}}
#include <amd_smi/amdsmi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <fstream>
#include <sstream>
#include <string>

#include "vgpu/minijson.h"

namespace {

minijson::Value g_fx;
bool g_loaded = false;
size_t g_event_cursor = 0;

const minijson::Value& gpus() { return g_fx["gpus"]; }

int idx(amdsmi_processor_handle h) { return (int)((uintptr_t)h) - 1; }

const minijson::Value* gpu(amdsmi_processor_handle h) {
  int i = idx(h);
  if (i < 0 || i >= (int)gpus().size()) return nullptr;
  return &gpus()[i];
}

void copy_str(char* dst, size_t n, const std::string& s) { snprintf(dst, n, "%s", s.c_str()); }

minijson::Value telemetry(amdsmi_processor_handle h) {
  minijson::Value v;
  const char* p = getenv("VGPU_FAKE_AMDSMI_TELEMETRY");
  if (!p) return v;
  std::ifstream f(p);
  if (!f) return v;
  std::stringstream ss;
  ss << f.rdbuf();
  minijson::Value all;
  if (!minijson::parse(ss.str(), all)) return v;
  return all[std::to_string(idx(h))];
}

}  // namespace

extern "C" {

amdsmi_status_t amdsmi_get_gpu_total_ecc_count(amdsmi_processor_handle h, amdsmi_error_count_t* ec) {
  if (!gpu(h)) return AMDSMI_STATUS_INVAL;
  auto t = telemetry(h);
  memset(ec, 0, sizeof(*ec));
  ec->uncorrectable_count = (uint64_t)t["ecc_ue"].num(0);
  ec->correctable_count = (uint64_t)t["ecc_ce"].num(0);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_power_info(amdsmi_processor_handle h, amdsmi_power_info_t* info) {
  if (!gpu(h)) return AMDSMI_STATUS_INVAL;
  auto t = telemetry(h);
  memset(info, 0, sizeof(*info));
  info->current_socket_power = (uint32_t)t["power"].num(0);
  info->socket_power = info->current_socket_power;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_temp_metric(amdsmi_processor_handle h, amdsmi_temperature_type_t type,
                                       amdsmi_temperature_metric_t, int64_t* out) {
  if (!gpu(h)) return AMDSMI_STATUS_INVAL;
  auto t = telemetry(h);
  const char* key = type == AMDSMI_TEMPERATURE_TYPE_EDGE ? "temp_edge"
                    : type == AMDSMI_TEMPERATURE_TYPE_HOTSPOT ? "temp_hotspot" : "temp_mem";
  *out = (int64_t)t[key].num(0);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_metrics_info(amdsmi_processor_handle h, amdsmi_gpu_metrics_t* m) {
  if (!gpu(h)) return AMDSMI_STATUS_INVAL;
  auto t = telemetry(h);
  memset(m, 0xff, sizeof(*m));  // "not supported" sentinel for every field we do not fill
  for (int l = 0; l < AMDSMI_MAX_NUM_XGMI_LINKS; ++l) m->xgmi_read_data_acc[l] = m->xgmi_write_data_acc[l] = 0;
  m->xgmi_read_data_acc[0] = (uint64_t)t["xgmi_read_kb"].num(0);
  m->xgmi_write_data_acc[0] = (uint64_t)t["xgmi_write_kb"].num(0);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_init(uint64_t) {
  const char* p = getenv("VGPU_FAKE_AMDSMI_JSON");
  if (!p) return AMDSMI_STATUS_INIT_ERROR;
  std::ifstream f(p);
  if (!f) return AMDSMI_STATUS_INIT_ERROR;
  std::stringstream ss;
  ss << f.rdbuf();
  if (!minijson::parse(ss.str(), g_fx)) return AMDSMI_STATUS_INIT_ERROR;
  g_loaded = true;
  g_event_cursor = 0;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_shut_down(void) {
  g_loaded = false;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_socket_handles(uint32_t* count, amdsmi_socket_handle* handles) {
  if (!g_loaded) return AMDSMI_STATUS_NOT_INIT;
  if (handles && *count >= 1) handles[0] = (amdsmi_socket_handle)(uintptr_t)1;
  *count = 1;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_processor_handles(amdsmi_socket_handle, uint32_t* count,
                                             amdsmi_processor_handle* handles) {
  uint32_t n = (uint32_t)gpus().size();
  if (handles)
    for (uint32_t i = 0; i < n && i < *count; ++i) handles[i] = (amdsmi_processor_handle)(uintptr_t)(i + 1);
  *count = n;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_processor_type(amdsmi_processor_handle h, processor_type_t* t) {
  *t = gpu(h) ? AMDSMI_PROCESSOR_TYPE_AMD_GPU : AMDSMI_PROCESSOR_TYPE_UNKNOWN;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_device_uuid(amdsmi_processor_handle h, unsigned int* len, char* uuid) {
  auto* g = gpu(h);
  if (!g) return AMDSMI_STATUS_INVAL;
  copy_str(uuid, *len, (*g)["uuid"].str());
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_device_bdf(amdsmi_processor_handle h, amdsmi_bdf_t* bdf) {
  auto* g = gpu(h);
  if (!g) return AMDSMI_STATUS_INVAL;
  unsigned dom = 0, bus = 0, dev = 0, fn = 0;
  sscanf((*g)["bdf"].str("0000:00:00.0").c_str(), "%x:%x:%x.%x", &dom, &bus, &dev, &fn);
  bdf->as_uint = 0;
  bdf->domain_number = dom;
  bdf->bus_number = bus;
  bdf->device_number = dev;
  bdf->function_number = fn;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_asic_info(amdsmi_processor_handle h, amdsmi_asic_info_t* info) {
  auto* g = gpu(h);
  if (!g) return AMDSMI_STATUS_INVAL;
  memset(info, 0, sizeof(*info));
  copy_str(info->market_name, sizeof info->market_name, (*g)["name"].str("AMD Instinct MI355X"));
  info->vendor_id = (uint32_t)(*g)["vendor"].num(0x1002);
  info->device_id = (uint64_t)(*g)["device_id"].num(0x75a3);
  info->num_of_compute_units = (uint32_t)(*g)["cus"].num(256);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_memory_total(amdsmi_processor_handle h, amdsmi_memory_type_t, uint64_t* v) {
  auto* g = gpu(h);
  if (!g) return AMDSMI_STATUS_INVAL;
  *v = (uint64_t)(*g)["vram"].num(309220868096.0);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_memory_usage(amdsmi_processor_handle h, amdsmi_memory_type_t, uint64_t* v) {
  auto* g = gpu(h);
  if (!g) return AMDSMI_STATUS_INVAL;
  *v = (uint64_t)(*g)["vram_used"].num(0);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_vram_usage(amdsmi_processor_handle h, amdsmi_vram_usage_t* info) {
  auto* g = gpu(h);
  if (!g) return AMDSMI_STATUS_INVAL;
  memset(info, 0, sizeof(*info));
  info->vram_total = (uint32_t)((uint64_t)(*g)["vram"].num(288.0 * (1ull << 30)) >> 20);
  info->vram_used = (uint32_t)((uint64_t)(*g)["vram_used"].num(0) >> 20);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_vram_info(amdsmi_processor_handle h, amdsmi_vram_info_t* info) {
  auto* g = gpu(h);
  if (!g) return AMDSMI_STATUS_INVAL;
  memset(info, 0, sizeof(*info));
  info->vram_type = AMDSMI_VRAM_TYPE_HBM3E;
  info->vram_size = (uint64_t)(*g)["vram"].num(288.0 * (1ull << 30)) >> 20;
  info->vram_bit_width = 8192;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_topo_numa_affinity(amdsmi_processor_handle h, int32_t* numa) {
  auto* g = gpu(h);
  if (!g) return AMDSMI_STATUS_INVAL;
  *numa = (int32_t)(*g)["numa"].num(0);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_topo_get_link_type(amdsmi_processor_handle a, amdsmi_processor_handle b,
                                          uint64_t* hops, amdsmi_link_type_t* type) {
  if (!gpu(a) || !gpu(b)) return AMDSMI_STATUS_INVAL;
  bool xgmi = g_fx["link"].str("xgmi") == "xgmi" &&
              (*gpu(a))["hive"].num(1) == (*gpu(b))["hive"].num(1);
  *hops = 1;
  *type = xgmi ? AMDSMI_LINK_TYPE_XGMI : AMDSMI_LINK_TYPE_PCIE;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_compute_partition(amdsmi_processor_handle h, char* out, uint32_t len) {
  auto* g = gpu(h);
  if (!g) return AMDSMI_STATUS_INVAL;
  copy_str(out, len, (*g)["partition"].str("SPX"));
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_memory_partition(amdsmi_processor_handle h, char* out, uint32_t len) {
  auto* g = gpu(h);
  if (!g) return AMDSMI_STATUS_INVAL;
  copy_str(out, len, (*g)["mem_partition"].str("NPS1"));
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_activity(amdsmi_processor_handle h, amdsmi_engine_usage_t* u) {
  auto* g = gpu(h);
  if (!g) return AMDSMI_STATUS_INVAL;
  memset(u, 0, sizeof(*u));
  u->gfx_activity = (uint32_t)(*g)["gfx"].num(0);
  u->umc_activity = (uint32_t)(*g)["umc"].num(0);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_process_list(amdsmi_processor_handle h, uint32_t* max,
                                            amdsmi_proc_info_t* list) {
  auto* g = gpu(h);
  if (!g) return AMDSMI_STATUS_INVAL;
  const auto& ps = (*g)["processes"];
  uint32_t n = (uint32_t)ps.size();
  for (uint32_t i = 0; i < n && i < *max; ++i) {
    memset(&list[i], 0, sizeof(list[i]));
    list[i].pid = (amdsmi_process_handle_t)ps[i]["pid"].num(0);
    list[i].memory_usage.vram_mem = (uint64_t)ps[i]["vram"].num(0);
    list[i].mem = list[i].memory_usage.vram_mem;
    list[i].cu_occupancy = (uint32_t)ps[i]["cu"].num(0);
    list[i].engine_usage.gfx = (uint64_t)ps[i]["gfx_ns"].num(0);
  }
  *max = n;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_kfd_info(amdsmi_processor_handle h, amdsmi_kfd_info_t* info) {
  auto* g = gpu(h);
  if (!g) return AMDSMI_STATUS_INVAL;
  memset(info, 0, sizeof(*info));
  info->kfd_id = (uint64_t)(*g)["kfd_id"].num(1000 + idx(h));
  info->node_id = (uint32_t)(idx(h) + 1);
  info->current_partition_id = (uint32_t)(*g)["partition_id"].num(0);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_enumeration_info(amdsmi_processor_handle h, amdsmi_enumeration_info_t* e) {
  auto* g = gpu(h);
  if (!g) return AMDSMI_STATUS_INVAL;
  memset(e, 0, sizeof(*e));
  e->drm_render = (uint32_t)(*g)["render"].num(128 + idx(h));
  e->drm_card = (uint32_t)(*g)["card"].num(idx(h));
  e->hip_id = (uint32_t)idx(h);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_xgmi_info(amdsmi_processor_handle h, amdsmi_xgmi_info_t* x) {
  auto* g = gpu(h);
  if (!g) return AMDSMI_STATUS_INVAL;
  memset(x, 0, sizeof(*x));
  x->xgmi_hive_id = (uint64_t)(*g)["hive"].num(1);
  x->index = (uint32_t)idx(h);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_init_gpu_event_notification(amdsmi_processor_handle) { return AMDSMI_STATUS_SUCCESS; }
amdsmi_status_t amdsmi_set_gpu_event_notification_mask(amdsmi_processor_handle, uint64_t) {
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_event_notification(int, uint32_t* num, amdsmi_evt_notification_data_t* data) {
  const auto& ev = g_fx["events"];
  uint32_t k = 0;
  while (g_event_cursor < ev.size() && k < *num) {
    const auto& e = ev[g_event_cursor++];
    data[k].processor_handle = (amdsmi_processor_handle)(uintptr_t)((int)e["gpu"].num(0) + 1);
    data[k].event = (amdsmi_evt_notification_type_t)(int)e["type"].num(0);
    copy_str(data[k].message, sizeof data[k].message, e["message"].str());
    ++k;
  }
  *num = k;
  return AMDSMI_STATUS_SUCCESS;
}

}  // extern "C"
