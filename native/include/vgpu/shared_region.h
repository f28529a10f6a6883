/*
 * vgpu shared region — the single source of truth for the per-container
 * accounting file that the in-container enforcement library (libvgpu.so)
 * and the node monitor (vgpu.monitor) both mmap(MAP_SHARED).
 *
 * Reference behaviour (what, not how):
 *   - cmd/vGPUmonitor/cudevshr.go:15-65   Go mirror of the closed-source
 *     shim's region (magic 19920718, 16 devices, 1024 process slots,
 *     per-process {context,module,buffer,offset,total} usage,
 *     recentKernel / utilizationSwitch / priority feedback words).
 *   - lib/nvidia/libvgpu.so: try_create_shrreg, fix_lock_shrreg,
 *     rm_quitted_process, set_task_pid.
 *
 * MI355X-first differences:
 *   - One robust, process-shared pthread mutex (EOWNERDEAD recovery) instead
 *     of a semaphore + timeout repair.
 *   - Per-device 256-bit CU masks (8 XCDs x 32 CUs) and per-device CU limits.
 *   - Host-resident ("virtual device memory") bytes and swap counters.
 *   - Every field the monitor may write is a naturally aligned 32/64-bit word
 *     accessed with __atomic builtins on both sides, and structural changes
 *     (slot claim/release) happen under the lock.
 *
 * Layout rules: fixed-size, no pointers, 8-byte aligned fields, explicit
 * padding.  The Python ctypes mirror (vgpu/monitor/region.py) asserts
 * sizeof/offsetof equality against vgpu_region_layout() at import.
 */
#ifndef VGPU_SHARED_REGION_H_
#define VGPU_SHARED_REGION_H_

#include <pthread.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VGPU_REGION_MAGIC 0x56475055u /* "VGPU" */
#define VGPU_REGION_VERSION 4u
#define VGPU_MAX_DEVICES 16
#define VGPU_MAX_PROCS 1024
#define VGPU_UUID_LEN 64
#define VGPU_CU_MASK_WORDS 4 /* 4 x 64 bit = 256 CUs (MI355X: 8 XCD x 32 CU) */

/* how a slot's host_pid was obtained */
#define VGPU_HOSTPID_UNVERIFIED 0 /* getpid()/NSpid: equals the host pid only outside a pid namespace */
#define VGPU_HOSTPID_KFD_DIFF 1   /* KFD proc-dir diff around our first /dev/kfd open (hostpid.cpp) */
#define VGPU_HOSTPID_MONITOR 2    /* node monitor (hostPID) matched NSpid + cgroup (vgpu/monitor/pids.py) */
#define VGPU_HOSTPID_HOST_NS 3    /* process runs in the host pid namespace */

/* vgpu_device_cfg_t.flags */
#define VGPU_DEV_FLAG_SUSPEND_EVICT 1u /* suspend (SIGUSR2) evicts the container's HBM (VGPU_SUSPEND_EVICT) */
/* Bits 16-31 of vgpu_device_cfg_t.flags: generation of the device plugin's
 * writes of cu_mask (vgpu_region_set_cu_mask bumps it).  The processes of a
 * container also write the mask (adaptive share claims); only a generation
 * change means the plugin reshaped the pool. */
#define VGPU_DEV_POOL_GEN_SHIFT 16

/* process slot status */
#define VGPU_PROC_FREE 0
#define VGPU_PROC_RUNNING 1
#define VGPU_PROC_SUSPENDED 2

/* per-device memory usage of one process, bytes */
typedef struct vgpu_dev_usage {
  uint64_t context_bytes; /* runtime context / queues charged at init        */
  uint64_t module_bytes;  /* code objects (hipModuleLoad*)                   */
  uint64_t buffer_bytes;  /* device allocations (hipMalloc & friends)        */
  uint64_t host_bytes;    /* oversubscribed bytes resident in host memory    */
  uint64_t total_bytes;   /* context + module + buffer (HBM-resident charge) */
  uint64_t peak_bytes;    /* high-water mark of total_bytes                  */
  uint64_t swap_out_bytes;/* pager: HBM -> host bytes moved                  */
  uint64_t swap_in_bytes; /* pager: host -> HBM bytes moved                  */
} vgpu_dev_usage_t;

typedef struct vgpu_proc_slot {
  int32_t pid;       /* pid as seen inside the container                     */
  int32_t host_pid;  /* pid in the host pid namespace (/proc/self/status NSpid) */
  int32_t status;    /* VGPU_PROC_*                                          */
  int32_t priority;  /* 0 = high, 1 = low                                    */
  int32_t host_pid_src; /* VGPU_HOSTPID_*                                    */
  int32_t reserved0;
  uint64_t start_ns; /* CLOCK_MONOTONIC at slot claim                        */
  uint64_t launches; /* kernel dispatches observed                           */
  uint64_t throttle_wait_ns; /* time spent blocked in the dispatch limiter   */
  uint64_t oom_events;       /* allocations refused by the cap               */
  uint64_t last_launch_ns;   /* CLOCK_MONOTONIC of the latest dispatch       */
  uint64_t pinned_host_bytes;/* page-locked host memory (hipHostMalloc & co.); not
                              * charged against the HBM cap, optionally capped by
                              * VGPU_PINNED_HOST_LIMIT                           */
  vgpu_dev_usage_t used[VGPU_MAX_DEVICES];
} vgpu_proc_slot_t;

typedef struct vgpu_device_cfg {
  char uuid[VGPU_UUID_LEN];
  uint64_t mem_limit;       /* bytes; 0 = unlimited                          */
  uint64_t mem_physical;    /* the container's physical HBM budget (bytes; 0 = whole device):
                             * virtual device memory keeps at most this much resident */
  uint32_t cu_limit;        /* percent of the device's CUs, 0 or >=100 = unlimited */
  uint32_t cu_total;        /* CUs on the physical device                    */
  uint64_t cu_mask[VGPU_CU_MASK_WORDS]; /* HSA logical CU mask; all-zero = no mask */
  /* Utilization of this container on the device as measured by the node
   * monitor (hostPID view of KFD cu_occupancy), consumed by the temporal
   * limiter when the shim has no verified host pid of its own. */
  volatile uint32_t busy_permille;      /* 0..1000 of the device's CUs            */
  uint32_t flags;                       /* VGPU_DEV_FLAG_*                          */
  volatile uint64_t busy_ns;            /* CLOCK_MONOTONIC of the sample; 0 = none */
} vgpu_device_cfg_t;

typedef struct vgpu_shared_region {
  uint32_t magic;
  uint32_t version;
  uint32_t struct_size;
  volatile int32_t initialized; /* 1 once limits were written               */
  union {
    pthread_mutex_t m;          /* PTHREAD_PROCESS_SHARED + ROBUST          */
    uint8_t raw[64];
  } lock;
  int32_t num_devices;
  int32_t oversubscribe;        /* 1 = virtual device memory enabled        */
  int32_t priority;             /* task priority of the container           */
  int32_t core_policy;          /* 0 default, 1 force, 2 disable            */
  /* feedback words written by the node monitor (vgpu.monitor.feedback)    */
  volatile int32_t recent_kernel;      /* shim sets 2 on launch; monitor decrements; <0 blocks launches */
  volatile int32_t utilization_switch; /* 1 = temporal throttling active    */
  volatile int32_t proc_num;           /* number of RUNNING/SUSPENDED slots */
  volatile int32_t monitor_seq;        /* bumped by each monitor observation */
  uint64_t create_ns;                  /* CLOCK_REALTIME ns of creation      */
  vgpu_device_cfg_t dev[VGPU_MAX_DEVICES];
  vgpu_proc_slot_t procs[VGPU_MAX_PROCS];
} vgpu_shared_region_t;

/* Layout descriptor exported by libvgpu so readers can check their mirror. */
typedef struct vgpu_region_layout {
  uint64_t region_size;
  uint64_t proc_slot_size;
  uint64_t dev_usage_size;
  uint64_t device_cfg_size;
  uint64_t off_lock;
  uint64_t off_num_devices;
  uint64_t off_recent_kernel;
  uint64_t off_dev;
  uint64_t off_procs;
  uint64_t mutex_size;
} vgpu_region_layout_t;

#ifdef __cplusplus
}  // extern "C"
#endif

#endif  // VGPU_SHARED_REGION_H_
