"""Host-PID resolution for container processes the shim could not verify.

Reference: cmd/vGPUmonitor/feedback.go:83-162 (`setHostPid`): the monitor maps
each container's processes to host pids through the cgroup driver's `tasks`
files (disabled in the reference, metrics.go:205-208).

The shim resolves its own host pid from a KFD process-directory diff under the
node-wide lock (native/shim/hostpid.cpp).  When that diff is ambiguous (two
processes of the node opened /dev/kfd in the same instant) the slot stays
VGPU_HOSTPID_UNVERIFIED, and a host-side purge cannot judge it, because a
container pid means nothing in the host namespace.  The monitor runs with
hostPID and finishes the job:

  * candidates = host processes whose /proc/<pid>/cgroup names the pod UID
    (cgroupfs `pod<uid>` or systemd `pod<uid with _>`), indexed by the
    innermost pid of their /proc/<pid>/status NSpid line;
  * a slot whose container pid has exactly one candidate gets it; with
    several (containers of one pod have separate pid namespaces, so pid 1 can
    repeat), the one whose start time is closest before the slot's claim;
  * the pid is written through the C library under the region lock with
    src = VGPU_HOSTPID_MONITOR, so the host-side purge
    (vgpu_region_purge(host_ns=1)) can now free the slot once it exits.
"""
from __future__ import annotations

import logging
import os
from collections import defaultdict

from .region import HOSTPID_MONITOR, HOSTPID_UNVERIFIED, PROC_FREE, AttachedRegion

log = logging.getLogger("vgpu.monitor.pids")

CLK_TCK = os.sysconf("SC_CLK_TCK") if hasattr(os, "sysconf") else 100


def _read(path: str) -> str:
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return ""


def nspid_chain(pid: int, proc_root: str = "/proc") -> list[int]:
    """NSpid: host pid first, innermost namespace pid last."""
    for line in _read(f"{proc_root}/{pid}/status").splitlines():
        if line.startswith("NSpid:"):
            try:
                return [int(x) for x in line.split()[1:]]
            except ValueError:
                return []
    return []


def start_ns(pid: int, proc_root: str = "/proc") -> int:
    """Process start time (ns since boot) from /proc/<pid>/stat field 22."""
    stat = _read(f"{proc_root}/{pid}/stat")
    try:
        fields = stat.rsplit(")", 1)[1].split()
        return int(fields[19]) * 1_000_000_000 // CLK_TCK
    except (IndexError, ValueError):
        return 0


def pod_uid_forms(uid: str) -> tuple[str, ...]:
    return (uid, uid.replace("-", "_"))


def candidates(pod_uid: str, proc_root: str = "/proc") -> dict[int, list[tuple[int, int]]]:
    """{container (innermost) pid: [(host pid, start ns), ...]} of the pod's processes."""
    forms = pod_uid_forms(pod_uid)
    out: dict[int, list[tuple[int, int]]] = defaultdict(list)
    try:
        entries = os.listdir(proc_root)
    except OSError:
        return out
    for e in entries:
        if not e.isdigit():
            continue
        cg = _read(f"{proc_root}/{e}/cgroup")
        if not cg or not any(f in cg for f in forms):
            continue
        chain = nspid_chain(int(e), proc_root)
        if len(chain) >= 1:
            out[chain[-1]].append((int(e), start_ns(int(e), proc_root)))
    return out


def resolve_region(region: AttachedRegion, pod_uid: str, proc_root: str = "/proc") -> int:
    """Resolve every unverified slot of one container region; returns how many
    slots got a host pid."""
    slots = [(i, s) for i, s in enumerate(region.r.procs)
             if s.status != PROC_FREE and s.host_pid_src == HOSTPID_UNVERIFIED]
    if not slots:
        return 0
    cand = candidates(pod_uid, proc_root)
    done = 0
    for i, s in slots:
        c = cand.get(s.pid, [])
        if not c:
            continue
        if len(c) > 1:
            # the process claimed its slot after it started: the closest start before the claim
            before = [x for x in c if x[1] <= s.start_ns] or c
            c = [max(before, key=lambda x: x[1])]
        host = c[0][0]
        if region.set_host_pid(i, s.pid, host, HOSTPID_MONITOR):
            done += 1
            log.info("slot %d: container pid %d is host pid %d (cgroup of pod %s)", i, s.pid, host, pod_uid)
    return done


def resolve_and_purge(regions: dict, proc_root: str = "/proc") -> tuple[int, int]:
    """One monitor pass over ContainerRegion objects (pathmonitor.py): resolve
    unverified host pids, then purge slots whose (host) process is gone."""
    resolved = purged = 0
    for cr in regions.values():
        resolved += resolve_region(cr.region, cr.pod_uid, proc_root)
        purged += max(cr.region.purge(host_ns=True), 0)
    return resolved, purged
