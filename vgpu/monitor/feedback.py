"""Priority feedback controller (every 5 s).

Reference: cmd/vGPUmonitor/feedback.go:197-255 (`Observe`): decrement every
region's recentKernel and count, per device and priority, the tasks that
launched recently; `CheckBlocking` (:164-177) — a higher-priority task is
active on one of my devices → recentKernel = -1, which blocks my launches in
the shim; `CheckPriority` (:180-195) — a higher-priority task, or another
task of my priority, is active → utilizationSwitch = 1 (throttling on), else 0.
Priority 0 is high, 1 is low.  Here all writes are atomic C calls on the
mapped region (the reference writes the shim's mmap with plain stores).

Suspend with eviction (reference libvgpu.so `suspend_all` /
`sig_swap_stub`): a container that opted in (device plugin --suspend-evict,
VGPU_SUSPEND_EVICT) and stays blocked by a higher-priority task for
SUSPEND_AFTER observations is sent SIGUSR2: its shim moves the container's
managed ranges to host memory, so the higher-priority pod can allocate that
HBM.  Once it has been unblocked for RESUME_AFTER observations it gets
SIGUSR1 and its pager brings the ranges back as they are used.  Hysteresis,
because an eviction moves the container's whole footprint over the host link.
"""
from __future__ import annotations

import signal
from collections import defaultdict

from .region import AttachedRegion

NUM_PRIORITIES = 2
SUSPEND_AFTER = 2   # observations blocked before an evicting suspend (2 x 5 s)
RESUME_AFTER = 1    # observations unblocked before the resume
_streak: dict[str, int] = {}  # region key -> +n blocked / -n unblocked observations in a row
SIGNAL_HOST_NS = True  # the monitor runs with hostPID: signal slots by their verified host pids


def _uuids(r: AttachedRegion) -> list[str]:
    return [d.uuid for d in r.devices() if d.uuid]


def observe(regions: dict[str, AttachedRegion]) -> dict[str, list[int]]:
    active: dict[str, list[int]] = defaultdict(lambda: [0] * NUM_PRIORITIES)
    for r in regions.values():
        if r.recent_kernel > 0:
            if r.decay_recent() > 0:
                p = min(max(r.priority, 0), NUM_PRIORITIES - 1)
                for u in _uuids(r):
                    active[u][p] += 1
    for key, r in regions.items():
        p = min(max(r.priority, 0), NUM_PRIORITIES - 1)
        uu = _uuids(r)
        blocking = any(active[u][q] > 0 for u in uu if u in active for q in range(p))
        if blocking:
            if r.recent_kernel >= 0:
                r.set_recent_kernel(-1)
        elif r.recent_kernel < 0:
            r.set_recent_kernel(0)
        _evicting_suspend(key, r, blocking)
        contended = any((any(active[u][q] > 0 for q in range(p)) or active[u][p] > 1)
                        for u in uu if u in active)
        want = 1 if contended else 0
        if r.utilization_switch != want:
            r.set_utilization_switch(want)
    return dict(active)


def _evicting_suspend(key: str, r: AttachedRegion, blocking: bool) -> None:
    if not r.suspend_evict:
        _streak.pop(key, None)
        return
    prev = _streak.get(key, 0)
    n = (max(prev, 0) + 1) if blocking else (min(prev, 0) - 1)
    _streak[key] = n
    if blocking and n >= SUSPEND_AFTER and not r.suspended():
        r.signal_all(signal.SIGUSR2, host_ns=SIGNAL_HOST_NS)
    elif not blocking and -n >= RESUME_AFTER and r.suspended():
        r.signal_all(signal.SIGUSR1, host_ns=SIGNAL_HOST_NS)
