/*
 * vgpu share board — one small mmap'd file per physical GPU in the node-wide
 * lock directory (/tmp/vgpulock, mounted into every vGPU container by the
 * device plugin's Allocate; reference: the "unified lock" directory,
 * pkg/device-plugin/nvidiadevice/nvinternal/plugin/server.go:357-369).
 *
 * It lets the temporal limiters of different pods on the same GPU charge
 * each other FAIR-SHARE GPU time instead of wall-clock busy time: while k
 * processes have work outstanding on the GPU, each is charged 1/k of the
 * elapsed time (processor-sharing virtual time, as in GPS/WFQ).  A pod alone
 * on the GPU is charged its full busy time; four busy pods are charged a
 * quarter each, so four 25 % pods run unthrottled at the GPU's full aggregate
 * rate while a lone 25 % pod is held to a quarter of the GPU.
 *
 * The reference's equivalent signal is NVML's per-process SM utilization
 * (libvgpu.so utilization_watcher / get_used_gpu_utilization, SURVEY.md §2.6
 * E1f); ROCm has no per-process busy-time counter for KFD user queues.
 *
 * Layout rules as in shared_region.h: fixed size, no pointers, robust
 * process-shared mutex, monitor-readable.
 */
#ifndef VGPU_BOARD_H_
#define VGPU_BOARD_H_

#include <pthread.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VGPU_BOARD_MAGIC 0x56424F44u /* "VBOD" */
#define VGPU_BOARD_VERSION 4u
#define VGPU_BOARD_SLOTS 128
#define VGPU_BOARD_STALE_NS 500000000ull /* a slot without heartbeat for 0.5 s is inactive */
/* auto_phase */
#define VGPU_AUTO_TEMPORAL 0      /* decided (or too few busy members): time sharing */
#define VGPU_AUTO_EXPLORE_T 1     /* measuring time sharing                          */
#define VGPU_AUTO_EXPLORE_S 2     /* measuring CU claims                             */
#define VGPU_AUTO_SPATIAL 3       /* decided: every member on CUs of its own         */
#define VGPU_AUTO_EXPLORE_T2 4    /* measuring time sharing again (A/B/A)             */
#define VGPU_AUTO_MEMO 16

typedef struct vgpu_board_slot {
  int32_t pid;                   /* pid inside the owner's container (0 = free) */
  int32_t host_pid;              /* host pid when known                         */
  volatile int32_t active;       /* 1 while the owner has work outstanding       */
  int32_t limit_pct;             /* the owner's compute limit (informational)    */
  volatile uint64_t heartbeat_ns;/* CLOCK_MONOTONIC, refreshed by the owner      */
  volatile uint64_t charged_ns;  /* fair-share GPU time charged so far           */
  volatile uint64_t busy_ns;     /* wall time with work outstanding so far       */
  double v_mark;                 /* board virtual time at the last charge        */
  uint64_t claim_ns;             /* CLOCK_MONOTONIC of the claim                 */
  /* Concurrency gate (VGPU_POOL_CONCURRENCY): at most N slots of the pool run
   * at once; the others wait, oldest first, and a runner yields after its
   * quantum when someone waits. */
  volatile int32_t running;      /* 1 while admitted to the running set          */
  int32_t reserved0;
  volatile uint64_t run_start_ns;   /* CLOCK_MONOTONIC of the last admission     */
  volatile uint64_t wait_since_ns;  /* waiting for admission since (0 = not)     */
  /* Adaptive share policy (VGPU_CU_SHARE=auto, limiter.cpp): CUs this slot
   * holds exclusively while its dispatches are too small to fill the GPU
   * (spatial mode); the auto pool members of the GPU run on the rest.
   * 4 x 64 bits = 256 CUs, same logical bit order as the region's cu_mask. */
  volatile uint64_t cu_claim[4];
  volatile int32_t auto_member;     /* 1: the slot runs the adaptive (auto) policy            */
  int32_t reserved2;
  volatile uint64_t auto_launches;  /* its dispatches so far (progress signal)                */
  uint64_t auto_mark;               /* auto_launches at the start of a measurement (leader)   */
  uint64_t auto_seen;               /* auto_launches at the leader's last look                */
  uint64_t auto_busy_ns;            /* when the leader last saw it progress                   */
  double auto_rate[3];              /* dispatches/s: time-shared [0], own CUs [1], time-shared [2] */
  double auto_hist[3];              /* dispatches/s in the last three steadiness buckets      */
  uint64_t auto_bucket_mark;        /* auto_launches at the current bucket's start            */
} vgpu_board_slot_t;

typedef struct vgpu_board {
  uint32_t magic;
  uint32_t version;
  uint32_t struct_size;
  volatile int32_t initialized;
  union {
    pthread_mutex_t m; /* PTHREAD_PROCESS_SHARED + ROBUST */
    uint8_t raw[64];
  } lock;
  double v;               /* virtual time (ns): advances at 1/max(1, n_active) */
  uint64_t last_ns;       /* CLOCK_MONOTONIC of the last advance              */
  int32_t n_active;       /* live active slots at the last advance            */
  int32_t reserved;
  /* Adaptive share policy (auto): a per-GPU A/B between time sharing and CU
   * claims, driven by the lowest live auto slot (limiter.cpp auto_step).   */
  volatile int32_t auto_phase;     /* VGPU_AUTO_*                                       */
  volatile int32_t auto_members;   /* busy members the current decision was made for    */
  volatile uint64_t auto_phase_ns; /* CLOCK_MONOTONIC when the phase began              */
  volatile int32_t auto_marked;    /* 1 once the phase's measurement window opened      */
  int32_t reserved3;
  volatile double auto_score;      /* mean own-CU / time-shared rate of the last A/B     */
  /* Decisions by busy-member count n (< VGPU_AUTO_MEMO): a count that comes back
   * within the re-explore period (pods pausing between phases of a job) takes
   * its earlier decision instead of a new A/B. */
  volatile int32_t auto_memo_phase[16];
  volatile uint64_t auto_memo_ns[16];   /* when decided, 0 = never              */
  volatile double auto_memo_score[16];
  volatile int32_t auto_pending_n;      /* a new busy-member count, acted on once */
  volatile int32_t auto_want;           /* an A/B is due once the members are steady (tries left) */
  volatile uint64_t auto_pending_ns;    /* it has held for the settle time        */
  volatile uint64_t auto_bucket_ns;     /* start of the current steadiness bucket  */
  vgpu_board_slot_t slot[VGPU_BOARD_SLOTS];
} vgpu_board_t;

#ifdef __cplusplus
}  // extern "C"
#endif

#endif  // VGPU_BOARD_H_
