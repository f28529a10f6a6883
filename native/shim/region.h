// Shared-region lifecycle: create/attach the mmap'd accounting file, robust
// process-shared locking, per-process slot claim/release, dead-process purge
// and usage queries.
//
// Reference behaviour: lib/nvidia/libvgpu.so `try_create_shrreg` (open + lseek
// + write + mmap + lockf + sem_init, limits from env, "Limit inconsistency"
// check), `rm_quitted_process`, `exit_handler`, `fix_lock_shrreg`
// (SURVEY.md §2.6 E1e); monitor side cmd/vGPUmonitor/cudevshr.go:112-127.
#pragma once

#include <string>

#include "vgpu/shared_region.h"

namespace vgpu {

struct DeviceLimits {
  int num_devices = 0;
  uint64_t mem_limit[VGPU_MAX_DEVICES] = {};
  uint64_t mem_physical[VGPU_MAX_DEVICES] = {};  // physical HBM budget (VGPU_DEVICE_MEMORY_PHYSICAL_<i>)
  uint32_t cu_limit[VGPU_MAX_DEVICES] = {};
  uint64_t cu_mask[VGPU_MAX_DEVICES][VGPU_CU_MASK_WORDS] = {};
  char uuid[VGPU_MAX_DEVICES][VGPU_UUID_LEN] = {};
  int oversubscribe = 0;
  int suspend_evict = 0;  // VGPU_SUSPEND_EVICT: managed ranges so a suspend can evict HBM
  int priority = 1;
  int core_policy = 0;  // 0 default, 1 force, 2 disable
};

// Read the env contract written by the device plugin's Allocate
// (vgpu/deviceplugin/allocate.py; reference server.go:335-353).
DeviceLimits limits_from_env();

// Map (creating if needed) the region file at `path`.  `path == nullptr`
// returns a process-private anonymous region.  On creation/reinit the limits
// are written from `lim` (may be null: attach only, used by the monitor).
vgpu_shared_region_t* region_map(const char* path, const DeviceLimits* lim, int* fd_out);
void region_unmap(vgpu_shared_region_t* r, int fd);

// Robust lock: recovers a mutex whose owner died (EOWNERDEAD) and purges
// that owner's slot.  Returns 0 on success.
int region_lock(vgpu_shared_region_t* r);
void region_unlock(vgpu_shared_region_t* r);

// Slot management (all take the lock internally).
int region_claim_slot(vgpu_shared_region_t* r, int pid, int host_pid, int priority);
void region_release_slot(vgpu_shared_region_t* r, int slot);
// Remove slots whose pid has exited. `host_ns` selects host_pid (monitor) vs pid.
int region_purge_dead(vgpu_shared_region_t* r, bool host_ns);
int region_purge_dead_locked(vgpu_shared_region_t* r, bool host_ns);

// Sum of HBM-resident charge on `dev` over live slots (caller holds lock or
// accepts a racy snapshot).
uint64_t region_device_used(const vgpu_shared_region_t* r, int dev);
uint64_t region_device_host_used(const vgpu_shared_region_t* r, int dev);

// PID of the calling process in the pid namespace that mounted /proc (first
// field of "NSpid:" in /proc/self/status).  Inside a normal container this is
// the container pid; the node monitor (hostPID) maps it to the host pid by
// scanning host /proc/*/status NSpid lists (vgpu/monitor/pids.py).
int host_pid_of_self();

void region_fill_layout(vgpu_region_layout_t* out);

}  // namespace vgpu
