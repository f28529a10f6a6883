/*
 * libvgpu_smi — device discovery / telemetry facade for the node agents.
 *
 * Reference analogues: the Hygon plugin's cgo libdrm_amdgpu + hwloc bindings
 * (pkg/device-plugin/hygon/dcu/amdgpu/amdgpu.go, hwloc/hwloc.go), the NVIDIA
 * plugin's NVML enumeration (pkg/device-plugin/nvidiadevice/nvinternal/rm/
 * nvml_manager.go) and the MLU cndev binding (pkg/device-plugin/mlu/cndev/).
 *
 * Backends: "amdsmi" (dlopen libamd_smi.so — or the fixture-driven fake of
 * the same ABI in tests), "sysfs" (KFD topology + PCI sysfs; root relocatable
 * with VGPU_SYSFS_ROOT for tests), "auto" (amdsmi, else sysfs).
 */
#ifndef VGPU_SMI_H_
#define VGPU_SMI_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VGPU_SMI_STR 64

typedef struct vgpu_smi_device {
  char uuid[VGPU_SMI_STR];
  char bdf[VGPU_SMI_STR];
  char name[VGPU_SMI_STR];
  char compute_partition[16];
  char memory_partition[16];
  uint64_t vram_total;
  uint64_t vram_used;
  uint64_t xgmi_hive;
  uint64_t device_id;
  uint32_t vendor_id;
  uint32_t cus;
  uint32_t num_xcc;
  int32_t numa_node;
  uint32_t render_minor;
  uint32_t card;
  uint32_t kfd_gpu_id;
  uint32_t index;
  uint32_t health;       /* 1 healthy */
  uint32_t gfx_activity; /* % */
  uint32_t umc_activity; /* % */
  uint32_t partition_id; /* compute partition of its physical GPU (0 in SPX) */
  uint32_t reserved[6];
} vgpu_smi_device_t;

typedef struct vgpu_smi_proc {
  uint32_t pid;
  uint32_t cu_occupancy;
  uint64_t vram_bytes;
  uint64_t gfx_ns;
} vgpu_smi_proc_t;

typedef struct vgpu_smi_event {
  int32_t device;
  int32_t type;   /* AMDSMI_EVT_NOTIF_* */
  char message[VGPU_SMI_STR * 2];
} vgpu_smi_event_t;

/* Health / host telemetry of one device (amdsmi: total ECC counts, power
 * info, temperature metrics, gpu_metrics xGMI accumulators; sysfs: RAS
 * *_err_count files and hwmon). Fields the backend cannot read stay 0. */
typedef struct vgpu_smi_telemetry {
  uint64_t ecc_correctable;
  uint64_t ecc_uncorrectable;
  uint64_t ecc_deferred;
  uint64_t xgmi_read_kb;   /* accumulated over all links */
  uint64_t xgmi_write_kb;
  uint32_t power_w;
  int32_t temp_edge_c;
  int32_t temp_hotspot_c;
  int32_t temp_mem_c;
  uint32_t valid;          /* bit 0 ecc, 1 power, 2 temperature, 3 xgmi */
  uint32_t reserved[7];
} vgpu_smi_telemetry_t;

#define VGPU_TELEM_ECC 1u
#define VGPU_TELEM_POWER 2u
#define VGPU_TELEM_TEMP 4u
#define VGPU_TELEM_XGMI 8u

/* link types */
#define VGPU_LINK_UNKNOWN 0
#define VGPU_LINK_PCIE 1
#define VGPU_LINK_XGMI 2

int vgpu_smi_open(const char* backend); /* device count, <0 on error */
const char* vgpu_smi_backend(void);
int vgpu_smi_count(void);
int vgpu_smi_get(int index, vgpu_smi_device_t* out);
int vgpu_smi_link(int a, int b, uint64_t* hops, int32_t* type);
int vgpu_smi_processes(int index, vgpu_smi_proc_t* out, int max);
int vgpu_smi_events(vgpu_smi_event_t* out, int max, int timeout_ms);
int vgpu_smi_telemetry(int index, vgpu_smi_telemetry_t* out);
void vgpu_smi_close(void);

#ifdef __cplusplus
}
#endif

#endif /* VGPU_SMI_H_ */
