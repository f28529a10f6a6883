"""Flat device state + the native scoring core (native/sched/score.cpp).

The scheduler keeps every registered device as one record of a numpy
structured array that mirrors `vgpu_sched_dev_t`.  The usage fields are
updated in place when a pod is added or removed, so a /filter call neither
rebuilds usage from the pod ledger nor copies it (reference getNodesUsage,
pkg/scheduler/scheduler.go:249-310, rebuilt it on every call).  The native
scorer walks the selected nodes' records with the reference semantics and
returns the chosen node and placements.  vgpu/scheduler/score.py stays the
readable Python definition; tests/test_scheduler.py checks that the two agree.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

from vgpu.api.resources import ContainerDevice, ContainerDeviceRequest, DeviceUsage

DEV_DTYPE = np.dtype([("used", "<i4"), ("count", "<i4"), ("usedmem", "<i8"), ("totalmem", "<i8"),
                      ("usedcores", "<i4"), ("totalcore", "<i4"), ("numa", "<i4"), ("health", "<i4"),
                      ("hive", "<i4"), ("type_id", "<i4")], align=True)
REQ_DTYPE = np.dtype([("nums", "<i4"), ("mem_percentage", "<i4"), ("memreq", "<i8"), ("coresreq", "<i4"),
                      ("ctr", "<i4")], align=True)
PICK_DTYPE = np.dtype([("dev", "<i4"), ("req", "<i4"), ("usedmem", "<i8"), ("usedcores", "<i4"),
                       ("pad", "<i4")], align=True)

_LIB = None


def load_lib():
    """libvgpu_sched.so, or None (the scheduler then scores in Python)."""
    global _LIB
    if _LIB is not None:
        return _LIB or None
    if os.environ.get("VGPU_SCHED_NATIVE", "1") == "0":
        _LIB = False
        return None
    from vgpu.native import LIB_DIR
    path = LIB_DIR / "libvgpu_sched.so"
    try:
        lib = ctypes.CDLL(str(path))
    except OSError:
        _LIB = False
        return None
    ds, rs, ps = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    lib.vgpu_sched_abi(ctypes.byref(ds), ctypes.byref(rs), ctypes.byref(ps))
    if (ds.value, rs.value, ps.value) != (DEV_DTYPE.itemsize, REQ_DTYPE.itemsize, PICK_DTYPE.itemsize):
        raise RuntimeError(f"libvgpu_sched ABI mismatch: {(ds.value, rs.value, ps.value)}")
    vp, ip, dp = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
    lib.vgpu_sched_filter.restype = ip
    lib.vgpu_sched_filter.argtypes = [vp, vp, vp, ip, vp, vp, ip, vp, ip, ip, ip, dp, ip, ip,
                                      ctypes.POINTER(dp), vp, ip, ctypes.POINTER(ip), vp]
    _LIB = lib
    return lib


@dataclass
class FilterResult:
    node: str | None
    score: float
    devices: list[list[ContainerDevice]]
    error: str = ""


class FlatState:
    """All registered devices in one array, node-contiguous."""

    def __init__(self, nodes: dict, pods: dict):
        self.node_names: list[str] = list(nodes)
        self.node_index = {n: i for i, n in enumerate(self.node_names)}
        ranks = sorted(range(len(self.node_names)), key=lambda i: self.node_names[i])
        self.node_rank = np.empty(len(self.node_names), dtype=np.int32)
        self.node_rank[np.asarray(ranks, dtype=np.int64)] = np.arange(len(ranks), dtype=np.int32)
        devs = [(n, d) for n in self.node_names for d in nodes[n].devices]
        self.dev_ids = [d.id for _, d in devs]
        # a device "type" for eligibility is (type string, advertised resource)
        self.dev_types = [(d.type, d.resource) for _, d in devs]
        self.types = sorted(set(self.dev_types))
        self.type_id = {t: i for i, t in enumerate(self.types)}
        self.hives: dict[str, int] = {}
        # Column-wise fill: one numpy assignment per field, not per record
        # (8 000 devices build in a few ms).
        self.arr = np.zeros(len(devs), dtype=DEV_DTYPE)
        if devs:
            self.arr["count"] = [d.count for _, d in devs]
            self.arr["totalmem"] = [d.devmem for _, d in devs]
            self.arr["totalcore"] = [d.devcore for _, d in devs]
            self.arr["numa"] = [d.numa for _, d in devs]
            self.arr["health"] = [1 if d.health else 0 for _, d in devs]
            self.arr["type_id"] = [self.type_id[(d.type, d.resource)] for _, d in devs]
            self.arr["hive"] = [self._hive(d.xgmi_hive) for _, d in devs]
        self.dev_index: dict[tuple[str, str], int] = {(n, d.id): i for i, (n, d) in enumerate(devs)}
        counts = [len(nodes[n].devices) for n in self.node_names]
        self.off = np.zeros(len(self.node_names) + 1, dtype=np.int32)
        if counts:
            self.off[1:] = np.cumsum(counts)
        self.apply_all(pods)

    def _hive(self, name: str) -> int:
        return self.hives.setdefault(name, len(self.hives) + 1) if name else 0

    def apply_all(self, pods: dict) -> None:
        """Add every pod's usage in one vectorised pass (np.add.at)."""
        idx, mem, cores = [], [], []
        for p in pods.values():
            for ctr in p.devices:
                for cd in ctr:
                    i = self.dev_index.get((p.node_id, cd.uuid))
                    if i is not None:
                        idx.append(i)
                        mem.append(cd.usedmem)
                        cores.append(cd.usedcores)
        if not idx:
            return
        ix = np.asarray(idx, dtype=np.int64)
        np.add.at(self.arr["used"], ix, 1)
        np.add.at(self.arr["usedmem"], ix, np.asarray(mem, dtype=np.int64))
        np.add.at(self.arr["usedcores"], ix, np.asarray(cores, dtype=np.int32))

    def update_device(self, node_id: str, d) -> bool:
        """Attribute change of a registered device, in place.  False when the
        change needs a rebuild (unknown device or a device type not in the table)."""
        i = self.dev_index.get((node_id, d.id))
        key = (d.type, d.resource)
        if i is None or key not in self.type_id:
            return False
        r = self.arr[i]
        r["count"], r["totalmem"], r["totalcore"] = d.count, d.devmem, d.devcore
        r["numa"], r["health"], r["hive"] = d.numa, 1 if d.health else 0, self._hive(d.xgmi_hive)
        r["type_id"] = self.type_id[key]
        self.dev_types[i] = key
        return True

    def apply(self, node_id: str, devices: list[list[ContainerDevice]], sign: int) -> None:
        for ctr in devices:
            for cd in ctr:
                i = self.dev_index.get((node_id, cd.uuid))
                if i is None:
                    continue
                r = self.arr[i]
                r["used"] += sign
                r["usedmem"] += sign * cd.usedmem
                r["usedcores"] += sign * cd.usedcores

    def filter(self, node_names: list[str] | None, nums: list[list[ContainerDeviceRequest]],
               check_type, annos: dict, xgmi_bind: bool, xgmi_weight: float, binpack_devices: bool,
               spread_nodes: bool) -> tuple[FilterResult, dict[str, str]]:
        lib = load_lib()
        failed: dict[str, str] = {}
        if node_names is None:
            sel = np.arange(len(self.node_names), dtype=np.int32)
        else:
            idx = []
            for n in node_names:
                i = self.node_index.get(n)
                if i is None:
                    failed[n] = "node unregistered"
                else:
                    idx.append(i)
            sel = np.asarray(idx, dtype=np.int32)
        reqs = [(c, k) for c, ctr in enumerate(nums) for k in ctr]
        rq = np.zeros(len(reqs), dtype=REQ_DTYPE)
        elig = np.zeros((max(len(reqs), 1), max(len(self.types), 1)), dtype=np.uint8)
        numa_bind = False
        for j, (c, k) in enumerate(reqs):
            rq[j] = (k.nums, k.mem_percentage, k.memreq, k.coresreq, c)
            for t, (tname, tres) in enumerate(self.types):
                stub = DeviceUsage(id="", index=0, used=0, count=0, usedmem=0, totalmem=0, usedcores=0,
                                   totalcore=0, type=tname, numa=0, health=True, resource=tres)
                ok, numa = check_type(annos, stub, k)
                elig[j, t] = 1 if ok else 0
                numa_bind |= bool(ok and numa)
        total_nums = int(sum(k.nums for _, k in reqs))
        picks = np.zeros(max(total_nums, 1), dtype=PICK_DTYPE)
        fits = np.zeros(max(len(sel), 1), dtype=np.uint8)
        score = ctypes.c_double()
        npicks = ctypes.c_int()
        ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        rc = lib.vgpu_sched_filter(ptr(self.arr), ptr(self.off), ptr(sel), len(sel), ptr(self.node_rank),
                                   ptr(rq), len(reqs), ptr(elig), len(self.types), int(numa_bind),
                                   int(xgmi_bind), float(xgmi_weight), int(binpack_devices), int(spread_nodes),
                                   ctypes.byref(score), ptr(picks), len(picks), ctypes.byref(npicks), ptr(fits))
        if rc == -2:
            return FilterResult(None, 0.0, [], "core limit can't exceed 100"), failed
        if rc < 0:
            for s, i in enumerate(sel):
                failed.setdefault(self.node_names[i], "no device fits the request")
            return FilterResult(None, 0.0, []), failed
        node = self.node_names[sel[rc]]
        out: list[list[ContainerDevice]] = [[] for _ in nums]
        for p in picks[:npicks.value]:
            c, k = reqs[int(p["req"])]
            out[c].append(ContainerDevice(uuid=self.dev_ids[int(p["dev"])], type=k.type,
                                          usedmem=int(p["usedmem"]), usedcores=int(p["usedcores"])))
        return FilterResult(node, float(score.value), out), failed
