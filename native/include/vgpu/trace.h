/* Per-process event trace of the enforcement library (VGPU_TRACE=<dir>).
 *
 * SURVEY.md §5 "Tracing / profiling": the reference has debug logs only; the
 * plan is a ring buffer of alloc / launch / throttle events with timestamps.
 * Each process that loads libvgpu.so with VGPU_TRACE set maps
 * <dir>/vgpu-trace-<pid>.bin: this header followed by `capacity` 32-byte
 * events.  Writers claim slots with one atomic add on `head` (the ring wraps;
 * `head` counts all events ever written) and publish a slot by storing its
 * `ts_ns` last.  Readers: vgpu/monitor/trace.py (ctypes mirror, size-checked).
 */
#ifndef VGPU_TRACE_H_
#define VGPU_TRACE_H_

#include <stdint.h>

#define VGPU_TRACE_MAGIC 0x56545243u /* "VTRC" */
#define VGPU_TRACE_VERSION 1u

enum vgpu_trace_type {
  VGPU_EV_ALLOC = 1,         /* a = bytes, b = kind (state.h AllocKind)       */
  VGPU_EV_FREE = 2,          /* a = bytes, b = kind                            */
  VGPU_EV_OOM = 3,           /* a = requested bytes, b = limit                 */
  VGPU_EV_LAUNCH = 4,        /* a = workgroups, b = 1 when exempt from limiter */
  VGPU_EV_THROTTLE = 5,      /* a = wait ns, b = workgroups                    */
  VGPU_EV_SUSPEND = 6,       /* a = wait ns                                    */
  VGPU_EV_PRIORITY_BLOCK = 7,/* a = wait ns                                    */
  VGPU_EV_QUEUE = 8,         /* a = queue address, b = CUs in its mask (0 = all) */
  VGPU_EV_GPU_TIME = 9,      /* a = fair-share GPU ns charged, b = wall ns busy */
  VGPU_EV_MIGRATE = 10,      /* a = bytes, b = (ns << 1) | 1 to HBM, 0 to host */
  VGPU_EV_COPY = 11,         /* peer copy: dev = destination, a = bytes, b = source device */
};

typedef struct vgpu_trace_event {
  uint64_t ts_ns; /* CLOCK_MONOTONIC; 0 = slot not yet published */
  uint32_t type;
  int32_t dev;
  uint64_t a;
  uint64_t b;
} vgpu_trace_event_t;

typedef struct vgpu_trace_header {
  uint32_t magic;
  uint32_t version;
  uint32_t header_size;
  uint32_t event_size;
  uint64_t capacity;
  uint64_t head; /* events ever claimed (atomic) */
  int32_t pid;
  int32_t host_pid;
  uint64_t start_ns;
  uint64_t reserved[2];
} vgpu_trace_header_t;

#ifdef __cplusplus
static_assert(sizeof(vgpu_trace_event_t) == 32, "trace event layout");
static_assert(sizeof(vgpu_trace_header_t) == 64, "trace header layout");
#endif

#endif /* VGPU_TRACE_H_ */
