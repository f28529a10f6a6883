"""Compute / memory partitions as the MIG analogue: which devices a node
advertises, under which resource names, with how much memory each.

Reference: the NVIDIA plugin's MIG strategies
(pkg/device-plugin/nvidiadevice/nvinternal/mig/mig.go:17-86,
rm/device_map.go:121-183, rm/nvml_devices.go:88-131):
  * none   — MIG devices are not exposed; whole GPUs only;
  * single — every GPU is MIG-partitioned the same way and each MIG device is
             advertised under the plain resource name;
  * mixed  — each MIG profile is its own resource (nvidia.com/mig-1g.10gb ...).

MI355X: a GPU in DPX / QPX / CPX compute-partition mode is 2 / 4 / 8 devices
to the OS (KFD nodes, render nodes) with 4 / 2 / 1 XCDs (128 / 64 / 32 CUs)
each.  The memory-partition mode (NPS1 / NPS2) decides how many HBM domains the
GPU's memory forms; the partitions of one domain share it, and each reports the
whole domain as its VRAM.  Advertising that per partition would promise the
same bytes 2–4 times over, so `--partition-memory split` (default) divides it:
a CPX partition on an NPS2 GPU gets 288 GB / 2 domains / 4 partitions = 36 GB.

Strategies (`--partition-strategy`):
  * none   — only unpartitioned (SPX) GPUs are advertised (amd.com/gpu);
  * single (default) — every device, partition or not, is an amd.com/gpu;
    the node must be uniform, devices in a minority mode are unhealthy;
  * mixed  — SPX GPUs are amd.com/gpu, partitions amd.com/gpu-dpx /
    amd.com/gpu-qpx / amd.com/gpu-cpx, each served by its own plugin socket.
The scheduler matches a request's count resource to the device's resource
(vgpu/device/amd.py), so a amd.com/gpu-cpx pod lands on CPX partitions only.
"""
from __future__ import annotations

import logging
from collections import Counter, defaultdict

from .discovery import Device

log = logging.getLogger("vgpu.deviceplugin.partitions")

STRATEGIES = ("none", "single", "mixed")
MODES = ("SPX", "DPX", "QPX", "CPX")


def mode_of(d: Device) -> str:
    m = (d.compute_partition or "SPX").upper()
    return m if m in MODES else "SPX"


def nps_domains(memory_partition: str) -> int:
    mp = (memory_partition or "NPS1").upper()
    return int(mp[3:]) if mp.startswith("NPS") and mp[3:].isdigit() else 1


def physical_key(d: Device) -> str:
    """Devices of one physical GPU share the PCI domain:bus:device (the
    partition is in the function number) -- or the uuid without a bdf."""
    if d.bdf and "." in d.bdf:
        return d.bdf.rsplit(".", 1)[0]
    return d.bdf or d.uuid


def resource_for(mode: str, base: str = "amd.com/gpu") -> str:
    return base if mode == "SPX" else f"{base}-{mode.lower()}"


def split_memory(devs: list[Device]) -> None:
    """Per partition: its NPS domain's memory / the partitions sharing it."""
    groups: dict[str, list[Device]] = defaultdict(list)
    for d in devs:
        groups[physical_key(d)].append(d)
    for g in groups.values():
        if len(g) < 2:
            continue
        share = max(1, len(g) // nps_domains(g[0].memory_partition))
        if share > 1:
            for d in g:
                d.vram_total //= share
                d.memory_shared_by = share


def plan(devs: list[Device], strategy: str = "single", base: str = "amd.com/gpu",
         memory: str = "split") -> tuple[dict[str, list[Device]], dict[str, str]]:
    """→ ({resource name: devices}, {uuid: why it is advertised unhealthy})."""
    if strategy not in STRATEGIES:
        raise ValueError(f"partition strategy must be one of {STRATEGIES}, got {strategy!r}")
    if memory == "split":
        split_memory(devs)
    bad: dict[str, str] = {}
    if strategy == "none":
        keep = [d for d in devs if mode_of(d) == "SPX"]
        for d in devs:
            if mode_of(d) != "SPX":
                log.info("partition strategy none: %s (%s partition %d) not advertised", d.uuid, mode_of(d),
                         d.partition_id)
        for d in keep:
            d.resource = base
        return {base: keep}, bad
    if strategy == "single":
        modes = Counter(mode_of(d) for d in devs)
        if len(modes) > 1:
            major = modes.most_common(1)[0][0]
            for d in devs:
                if mode_of(d) != major:
                    bad[d.uuid] = f"partition strategy single: {mode_of(d)} on a {major} node"
        for d in devs:
            d.resource = base
        return {base: list(devs)}, bad
    out: dict[str, list[Device]] = defaultdict(list)
    for d in devs:
        d.resource = resource_for(mode_of(d), base)
        out[d.resource].append(d)
    return dict(out), bad


def socket_name(resource: str, base: str = "amd.com/gpu") -> str:
    """amd.com/gpu → amd-vgpu.sock, amd.com/gpu-cpx → amd-vgpu-cpx.sock."""
    return "amd-vgpu.sock" if resource == base else f"amd-vgpu-{resource.rsplit('-', 1)[-1]}.sock"
