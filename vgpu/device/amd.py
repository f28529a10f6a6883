"""AMD Instinct (MI355X) device policy: resource parsing with the reference's
defaults, GPU-type allow/deny lists, NUMA binding and xGMI binding.

Reference: pkg/device/nvidia/device.go:15-23 (annotation consts), :41-47
(ParseConfig resource-name flags), :49-60 (MutateAdmission injects the task
priority env), :62-94 (checkGPUtype: comma-separated, case-insensitive
substring allow/deny), :96-105 (assertNuma), :107-112 (CheckType),
:114-175 (GenerateResourceRequests: mem% sentinel 101, DefaultMem fallback,
DefaultCores).  Hygon DCU names (pkg/device/hygon/device.go:15-22) are accepted
as aliases — Hygon's DCU is the AMD-lineage device in the reference.
"""
from __future__ import annotations

import argparse

from vgpu import config
from vgpu.api import resources as R
from vgpu.api.env import ENV_PRIORITY
from vgpu.api.resources import ContainerDeviceRequest, DeviceUsage
from vgpu.k8s.objects import limit_or_request, parse_quantity

from .base import Devices


def check_gpu_type(annos: dict, card_type: str) -> bool:
    inuse = annos.get(R.ANN_USE_GPUTYPE)
    if inuse is not None:
        return any(v.strip().upper() in card_type.upper() for v in inuse.split(","))
    nouse = annos.get(R.ANN_NOUSE_GPUTYPE)
    if nouse is not None:
        return not any(v.strip().upper() in card_type.upper() for v in nouse.split(","))
    return True


def _parse_bool(v) -> bool | None:
    if v is None:
        return None
    s = str(v)
    if s in ("1", "t", "T", "TRUE", "true", "True"):
        return True
    if s in ("0", "f", "F", "FALSE", "false", "False"):
        return False
    return None


def assert_numa(annos: dict) -> bool:
    return bool(_parse_bool(annos.get(R.ANN_NUMA_BIND)))


def assert_xgmi(annos: dict) -> bool:
    return bool(_parse_bool(annos.get(R.ANN_XGMI_BIND)))


class AMDDevices(Devices):
    vendor = R.VENDOR
    handshake_annotation = R.NODE_HANDSHAKE
    register_annotation = R.NODE_REGISTER

    def __init__(self):
        self.resource_count = R.RESOURCE_COUNT
        self.resource_mem = R.RESOURCE_MEM
        self.resource_mem_pct = R.RESOURCE_MEM_PERCENTAGE
        self.resource_cores = R.RESOURCE_CORES
        self.resource_priority = R.RESOURCE_PRIORITY

    def parse_config(self, ap: argparse.ArgumentParser) -> None:
        ap.add_argument("--resource-name", default=R.RESOURCE_COUNT)
        ap.add_argument("--resource-mem", default=R.RESOURCE_MEM)
        ap.add_argument("--resource-mem-percentage", default=R.RESOURCE_MEM_PERCENTAGE)
        ap.add_argument("--resource-cores", default=R.RESOURCE_CORES)
        ap.add_argument("--resource-priority", default=R.RESOURCE_PRIORITY)

    def apply_config(self, ns: argparse.Namespace) -> None:
        self.resource_count = getattr(ns, "resource_name", self.resource_count)
        self.resource_mem = getattr(ns, "resource_mem", self.resource_mem)
        self.resource_mem_pct = getattr(ns, "resource_mem_percentage", self.resource_mem_pct)
        self.resource_cores = getattr(ns, "resource_cores", self.resource_cores)
        self.resource_priority = getattr(ns, "resource_priority", self.resource_priority)

    def _get(self, ctr: dict, name: str):
        v = limit_or_request(ctr, name)
        if v is None:
            for alias, canon in R.RESOURCE_ALIASES.items():
                if canon == name:
                    v = limit_or_request(ctr, alias)
                    if v is not None:
                        break
        return v

    def count_resources(self) -> list[str]:
        """amd.com/gpu plus the compute-partition resources of a node running the
        mixed partition strategy (vgpu/deviceplugin/partitions.py)."""
        return [self.resource_count] + [f"{self.resource_count}-{m}" for m in R.PARTITION_SUFFIXES]

    def _count(self, ctr: dict) -> tuple[str, object]:
        for name in self.count_resources():
            v = self._get(ctr, name)
            if v is not None:
                return name, v
        return self.resource_count, None

    def mutate_admission(self, ctr: dict) -> bool:
        lim = (ctr.get("resources") or {}).get("limits") or {}
        prio = lim.get(self.resource_priority)
        if prio is not None:
            env = ctr.setdefault("env", [])
            env.append({"name": ENV_PRIORITY, "value": str(parse_quantity(prio))})
        return self._count(ctr)[1] is not None

    def check_type(self, annos: dict, dev: DeviceUsage, req: ContainerDeviceRequest):
        if req.type == self.vendor:
            # the count resource must be the one the device is advertised under
            # (a amd.com/gpu-cpx request only fits CPX partitions of a mixed node)
            ok = check_gpu_type(annos, dev.type) and dev.resource == req.resource
            return True, ok, assert_numa(annos)
        return False, False, False

    def generate_resource_requests(self, ctr: dict) -> ContainerDeviceRequest:
        res, v = self._count(ctr)
        n = parse_quantity(v)
        if v is None or n is None:
            return ContainerDeviceRequest(nums=0)
        memnum = parse_quantity(self._get(ctr, self.resource_mem)) or 0
        mempct = parse_quantity(self._get(ctr, self.resource_mem_pct))
        mempct = R.MEM_PERCENT_UNSET if mempct is None else mempct
        if mempct == R.MEM_PERCENT_UNSET and memnum == 0:
            if config.SCHEDULER.default_mem:
                memnum = config.SCHEDULER.default_mem
            else:
                mempct = 100
        cores = parse_quantity(self._get(ctr, self.resource_cores))
        corenum = config.SCHEDULER.default_cores if cores is None else cores
        return ContainerDeviceRequest(nums=int(n), type=self.vendor, memreq=int(memnum),
                                      mem_percentage=int(mempct), coresreq=int(corenum), resource=res)
