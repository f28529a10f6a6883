"""Priority feedback controller (every 5 s).

Reference: cmd/vGPUmonitor/feedback.go:197-255 (`Observe`): decrement every
region's recentKernel and count, per device and priority, the tasks that
launched recently; `CheckBlocking` (:164-177) — a higher-priority task is
active on one of my devices → recentKernel = -1, which blocks my launches in
the shim; `CheckPriority` (:180-195) — a higher-priority task, or another
task of my priority, is active → utilizationSwitch = 1 (throttling on), else 0.
Priority 0 is high, 1 is low.  Here all writes are atomic C calls on the
mapped region (the reference writes the shim's mmap with plain stores).
"""
from __future__ import annotations

from collections import defaultdict

from .region import AttachedRegion

NUM_PRIORITIES = 2


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
    for r in regions.values():
        p = min(max(r.priority, 0), NUM_PRIORITIES - 1)
        uu = _uuids(r)
        blocking = any(active[u][q] > 0 for u in uu if u in active for q in range(p))
        if blocking:
            if r.recent_kernel >= 0:
                r.set_recent_kernel(-1)
        elif r.recent_kernel < 0:
            r.set_recent_kernel(0)
        contended = any((any(active[u][q] > 0 for q in range(p)) or active[u][p] > 1)
                        for u in uu if u in active)
        want = 1 if contended else 0
        if r.utilization_switch != want:
            r.set_utilization_switch(want)
    return dict(active)
