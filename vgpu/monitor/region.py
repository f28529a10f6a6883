"""ctypes mirror of native/include/vgpu/shared_region.h and an attached view
of one container's region.

Reference: cmd/vGPUmonitor/cudevshr.go:15-65 (Go mirror of the shim struct,
magic 19920718), :112-127 (mmap MAP_SHARED).  Unlike the reference, the mirror
is checked field-by-field against the C layout (`vgpu_region_layout`) at
attach time, every structural write goes through the C library under the
region's robust lock, and the feedback words are written with atomics.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

from vgpu.native import load_capi, region_layout

MAX_DEVICES = 16
MAX_PROCS = 1024
UUID_LEN = 64
CU_WORDS = 4
MAGIC = 0x56475055
VERSION = 4
PROC_FREE, PROC_RUNNING, PROC_SUSPENDED = 0, 1, 2
DEV_FLAG_SUSPEND_EVICT = 1  # shared_region.h VGPU_DEV_FLAG_SUSPEND_EVICT
# slot.host_pid_src (how the host pid was obtained)
HOSTPID_UNVERIFIED, HOSTPID_KFD_DIFF, HOSTPID_MONITOR, HOSTPID_HOST_NS = 0, 1, 2, 3


class DevUsage(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "context_bytes", "module_bytes", "buffer_bytes", "host_bytes", "total_bytes", "peak_bytes",
        "swap_out_bytes", "swap_in_bytes")]


class ProcSlot(ctypes.Structure):
    _fields_ = [("pid", ctypes.c_int32), ("host_pid", ctypes.c_int32), ("status", ctypes.c_int32),
                ("priority", ctypes.c_int32), ("host_pid_src", ctypes.c_int32), ("reserved0", ctypes.c_int32),
                ("start_ns", ctypes.c_uint64), ("launches", ctypes.c_uint64),
                ("throttle_wait_ns", ctypes.c_uint64), ("oom_events", ctypes.c_uint64),
                ("last_launch_ns", ctypes.c_uint64), ("pinned_host_bytes", ctypes.c_uint64),
                ("used", DevUsage * MAX_DEVICES)]


class DeviceCfg(ctypes.Structure):
    _fields_ = [("uuid", ctypes.c_char * UUID_LEN), ("mem_limit", ctypes.c_uint64),
                ("mem_physical", ctypes.c_uint64), ("cu_limit", ctypes.c_uint32),
                ("cu_total", ctypes.c_uint32), ("cu_mask", ctypes.c_uint64 * CU_WORDS),
                ("busy_permille", ctypes.c_uint32), ("flags", ctypes.c_uint32), ("busy_ns", ctypes.c_uint64)]


class Region(ctypes.Structure):
    _fields_ = [("magic", ctypes.c_uint32), ("version", ctypes.c_uint32), ("struct_size", ctypes.c_uint32),
                ("initialized", ctypes.c_int32), ("lock", ctypes.c_uint8 * 64),
                ("num_devices", ctypes.c_int32), ("oversubscribe", ctypes.c_int32),
                ("priority", ctypes.c_int32), ("core_policy", ctypes.c_int32),
                ("recent_kernel", ctypes.c_int32), ("utilization_switch", ctypes.c_int32),
                ("proc_num", ctypes.c_int32), ("monitor_seq", ctypes.c_int32),
                ("create_ns", ctypes.c_uint64), ("dev", DeviceCfg * MAX_DEVICES),
                ("procs", ProcSlot * MAX_PROCS)]


def check_layout() -> None:
    lay = region_layout()
    mine = {
        "region_size": ctypes.sizeof(Region), "proc_slot_size": ctypes.sizeof(ProcSlot),
        "dev_usage_size": ctypes.sizeof(DevUsage), "device_cfg_size": ctypes.sizeof(DeviceCfg),
        "off_lock": Region.lock.offset, "off_num_devices": Region.num_devices.offset,
        "off_recent_kernel": Region.recent_kernel.offset, "off_dev": Region.dev.offset,
        "off_procs": Region.procs.offset,
    }
    bad = {k: (v, lay[k]) for k, v in mine.items() if lay[k] != v}
    if bad:
        raise RuntimeError(f"shared region layout mismatch (python, C): {bad}")


@dataclass
class DeviceView:
    index: int
    uuid: str
    mem_limit: int
    cu_limit: int
    cu_mask: int
    used: int          # HBM-resident charge over live processes
    host_used: int     # oversubscribed bytes in host memory
    context: int
    module: int
    buffer: int
    swap_in: int
    swap_out: int
    busy_permille: int = 0   # fair-share GPU time of the last limiter window (shim-published)
    busy_ns: int = 0
    flags: int = 0           # DEV_FLAG_*


class AttachedRegion:
    """A container's region mapped into this process."""

    def __init__(self, path: str, create: bool = False):
        self.lib = load_capi()
        check_layout()
        self.path = path
        ptr = self.lib.vgpu_region_create(path.encode()) if create else self.lib.vgpu_region_attach(path.encode())
        if not ptr:
            raise FileNotFoundError(f"cannot attach shared region {path}")
        self.ptr = ptr
        self.r = Region.from_address(ptr)

    def close(self) -> None:
        if self.ptr:
            self.lib.vgpu_region_detach(self.ptr)
            self.ptr = None

    # ---- reads (racy snapshots are fine for metrics) --------------------------------
    def live_slots(self) -> list[ProcSlot]:
        return [s for s in self.r.procs if s.status != PROC_FREE]

    def devices(self) -> list[DeviceView]:
        out = []
        slots = self.live_slots()
        n = self.r.num_devices if 0 < self.r.num_devices <= MAX_DEVICES else 0
        for i in range(n):
            d = self.r.dev[i]
            mask = 0
            for w in range(CU_WORDS):
                mask |= d.cu_mask[w] << (64 * w)
            agg = {f: sum(getattr(s.used[i], f) for s in slots) for f, _ in DevUsage._fields_}
            out.append(DeviceView(i, d.uuid.decode(errors="replace"), d.mem_limit, d.cu_limit, mask,
                                  agg["total_bytes"], agg["host_bytes"], agg["context_bytes"],
                                  agg["module_bytes"], agg["buffer_bytes"], agg["swap_in_bytes"],
                                  agg["swap_out_bytes"], d.busy_permille, d.busy_ns, d.flags))
        return out

    @property
    def priority(self) -> int:
        return self.r.priority

    @property
    def suspend_evict(self) -> bool:
        """The container opted into suspend-with-eviction (VGPU_SUSPEND_EVICT)."""
        n = self.r.num_devices if 0 < self.r.num_devices <= MAX_DEVICES else 0
        return any(self.r.dev[i].flags & DEV_FLAG_SUSPEND_EVICT for i in range(n))

    def suspended(self) -> bool:
        """Any live process of the container is suspended (SIGUSR2)."""
        return any(s.status == PROC_SUSPENDED for s in self.live_slots())

    @property
    def recent_kernel(self) -> int:
        return self.r.recent_kernel

    @property
    def utilization_switch(self) -> int:
        return self.r.utilization_switch

    # ---- writes (through the C library) --------------------------------------------
    def decay_recent(self) -> int:
        return self.lib.vgpu_region_decay_recent(self.ptr)

    def set_recent_kernel(self, v: int) -> None:
        self.lib.vgpu_region_set_feedback(self.ptr, v, -1, 1)

    def set_utilization_switch(self, v: int) -> None:
        self.lib.vgpu_region_set_feedback(self.ptr, 0, v, 0)

    def set_cu_mask(self, dev: int, mask: int) -> None:
        words = (ctypes.c_uint64 * CU_WORDS)(*[(mask >> (64 * w)) & ((1 << 64) - 1) for w in range(CU_WORDS)])
        self.lib.vgpu_region_set_cu_mask(self.ptr, dev, words)

    def set_host_pid(self, slot: int, pid: int, host_pid: int, src: int = HOSTPID_MONITOR) -> bool:
        """Record a host pid the monitor resolved (only for a slot that still
        holds container pid `pid` and is unverified)."""
        return self.lib.vgpu_region_set_host_pid(self.ptr, slot, pid, host_pid, src) == 1

    def purge(self, host_ns: bool = True) -> int:
        return self.lib.vgpu_region_purge(self.ptr, 1 if host_ns else 0)

    def signal_all(self, sig: int, host_ns: bool = True) -> int:
        return self.lib.vgpu_region_signal_all(self.ptr, sig, 1 if host_ns else 0)
