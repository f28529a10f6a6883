"""Node/device scoring and bin-packing.

Reference semantics (pkg/scheduler/score.go):
  * devices of a node sorted by (NUMA, free slots) ascending and walked from the
    end — most-free device first (:45-50, :86-152);
  * per device: slot available, memory (absolute MiB or % of the device),
    cores, `gpucores == 100` needs an unused device, `gpucores == 0` cannot land
    on a device whose cores are fully allocated, core request > 100 is an error,
    vendor type / allow-deny list, `numa-bind` keeps every device of a container
    on one NUMA node (:86-152);
  * node score = Σcount/Σfree + (ndev − nreq) summed over containers (:154-181);
    the extender picks the highest (spread inside a node, pack across nodes).

MI355X additions (all default-neutral, so reference placements are unchanged
for single-GPU pods):
  * `amd.com/xgmi-bind: "true"` keeps a multi-GPU container inside one xGMI hive
    (same mechanism as numa-bind);
  * multi-GPU containers get `xgmi_weight` bonus per extra device sharing the
    hive of the first (RCCL rings over xGMI instead of PCIe);
  * `gpu_scheduler_policy=binpack` walks least-free devices first (pack pods
    onto already-shared GPUs, keep whole GPUs free for exclusive jobs).
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field

from vgpu import config
from vgpu.api.resources import ContainerDevice, ContainerDeviceRequest, DeviceUsage, MEM_PERCENT_UNSET
from vgpu.device.amd import assert_xgmi
from vgpu.device.base import get_devices


@dataclass
class NodeUsage:
    devices: list[DeviceUsage] = field(default_factory=list)


@dataclass
class NodeScore:
    node_id: str
    score: float = 0.0
    devices: list[list[ContainerDevice]] = field(default_factory=list)


class FitError(Exception):
    pass


def _sort_key(d: DeviceUsage, policy: str):
    """Reference order is (NUMA, free slots); ties are broken by free memory so
    that mixed-size requests spread by HBM too (the reference leaves the tie to
    the previous order, which strands 144 GB requests on already-full GPUs)."""
    free = d.count - d.used
    free_mem = d.totalmem - d.usedmem
    if policy == "spread":
        return (d.numa, free, free_mem)
    return (d.numa, -free, -free_mem)


def check_type(annos: dict, d: DeviceUsage, req: ContainerDeviceRequest) -> tuple[bool, bool]:
    """General vendor check (device type must contain the request vendor), then
    the vendor's own CheckType (reference score.go:71-84)."""
    if req.type not in d.type:
        return False, False
    for dev in get_devices().values():
        found, ok, numa = dev.check_type(annos, d, req)
        if found:
            return ok, numa
    return False, False


def fit_in_certain_device(node: NodeUsage, req: ContainerDeviceRequest, annos: dict
                          ) -> tuple[bool, list[ContainerDevice]]:
    k = copy.copy(req)
    origin = k.nums
    prev_numa = None
    prev_hive = None
    xgmi = assert_xgmi(annos) and origin > 1
    tmp: list[ContainerDevice] = []
    for i in range(len(node.devices) - 1, -1, -1):
        d = node.devices[i]
        ok, numa = check_type(annos, d, k)
        if not ok:
            continue
        if not d.health:
            continue
        if numa and prev_numa != d.numa:
            k.nums = origin
            prev_numa = d.numa
            tmp = []
        if xgmi and prev_hive != d.xgmi_hive:
            k.nums = origin
            prev_hive = d.xgmi_hive
            tmp = []
        if d.count <= d.used:
            continue
        if k.coresreq > 100:
            raise FitError("core limit can't exceed 100")
        memreq = k.memreq if k.memreq > 0 else 0
        if k.mem_percentage != MEM_PERCENT_UNSET and k.memreq == 0:
            memreq = d.totalmem * k.mem_percentage // 100
        if d.totalmem - d.usedmem < memreq:
            continue
        if d.totalcore - d.usedcores < k.coresreq:
            continue
        # gpucores=100 asks for the whole device
        if d.totalcore == 100 and k.coresreq == 100 and d.used > 0:
            continue
        # a best-effort (cores=0) job cannot land on a device whose cores are all allocated
        if d.totalcore != 0 and d.usedcores == d.totalcore and k.coresreq == 0:
            continue
        if k.nums > 0:
            k.nums -= 1
            tmp.append(ContainerDevice(uuid=d.id, type=k.type, usedmem=memreq,
                                       usedcores=k.coresreq, idx=i))
        if k.nums == 0:
            return True, tmp
    return False, tmp


def fit_in_devices(node: NodeUsage, reqs: list[ContainerDeviceRequest], annos: dict
                   ) -> tuple[bool, float, list[ContainerDevice]]:
    policy = config.SCHEDULER.gpu_scheduler_policy
    devs: list[ContainerDevice] = []
    total = 0
    free = 0
    sums = 0
    bonus = 0.0
    for k in reqs:
        sums += k.nums
        if k.nums > len(node.devices):
            return False, 0.0, devs
        node.devices.sort(key=lambda d: _sort_key(d, policy))
        fit, tmp = fit_in_certain_device(node, k, annos)
        if not fit:
            return False, 0.0, devs
        hives = [node.devices[c.idx].xgmi_hive for c in tmp]
        if len(tmp) > 1 and hives[0]:
            bonus += config.SCHEDULER.xgmi_weight * sum(h == hives[0] for h in hives[1:]) / (len(tmp) - 1)
        for c in tmp:
            d = node.devices[c.idx]
            total += d.count
            free += d.count - d.used
            d.used += 1
            d.usedcores += c.usedcores
            d.usedmem += c.usedmem
        devs.extend(tmp)
    score = (total / free if free else float(total)) + (len(node.devices) - sums) + bonus
    return True, score, devs


def calc_score(nodes: dict[str, NodeUsage], nums: list[list[ContainerDeviceRequest]],
               annos: dict) -> list[NodeScore]:
    """Score every node; nodes that cannot fit every container are dropped.
    `nodes` is mutated (usage of the tentative placement) — pass copies."""
    res = []
    for node_id, node in nodes.items():
        sc = NodeScore(node_id=node_id)
        for n in nums:
            if sum(k.nums for k in n) == 0:
                sc.devices.append([])
                continue
            fit, s, devs = fit_in_devices(node, n, annos)
            if not fit:
                break
            sc.devices.append(devs)
            sc.score += s
        if len(sc.devices) == len(nums):
            res.append(sc)
    return res


def pick_node(scores: list[NodeScore]) -> NodeScore | None:
    if not scores:
        return None
    if config.SCHEDULER.node_scheduler_policy == "spread":
        return min(scores, key=lambda s: (s.score, s.node_id))
    return max(scores, key=lambda s: (s.score, s.node_id))
