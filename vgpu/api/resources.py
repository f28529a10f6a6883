"""Pod-facing API: extended resource names, annotations and the node/pod
annotation keys (wire-compatible with the reference's text formats).

Reference: pkg/device/nvidia/device.go:15-23 (annotation consts), :41-47
(resource-name flags), pkg/util/types.go:26-35 (pod annotation keys),
pkg/device/devices.go:27-34 (handshake/register registry).

The MI355X stack exposes one vendor, ``amd.com``.  Hygon's ``hygon.com/dcu*``
names (the AMD-lineage device in the reference, pkg/device/hygon/device.go:15-22)
are accepted as aliases so existing pod specs keep scheduling.
"""
from __future__ import annotations

from dataclasses import dataclass, field

VENDOR = "AMD"
DEVICE_TYPE_PREFIX = "AMD-"          # device type string, e.g. "AMD-MI355X"

# ---- extended resources (per container limits) --------------------------------
RESOURCE_COUNT = "amd.com/gpu"
# compute-partition count resources of a mixed-strategy node: amd.com/gpu-cpx ...
PARTITION_SUFFIXES = ("dpx", "qpx", "cpx")
RESOURCE_MEM = "amd.com/gpumem"
RESOURCE_MEM_PERCENTAGE = "amd.com/gpumem-percentage"
RESOURCE_CORES = "amd.com/gpucores"
RESOURCE_PRIORITY = "amd.com/priority"

# Aliases accepted on input (Hygon DCU names from the reference).
RESOURCE_ALIASES = {
    "hygon.com/dcunum": RESOURCE_COUNT,
    "hygon.com/dcumem": RESOURCE_MEM,
    "hygon.com/dcucores": RESOURCE_CORES,
}

# ---- pod annotations (user-set) ---------------------------------------------------
ANN_USE_GPUTYPE = "amd.com/use-gputype"
ANN_NOUSE_GPUTYPE = "amd.com/nouse-gputype"
ANN_NUMA_BIND = "amd.com/numa-bind"
ANN_XGMI_BIND = "amd.com/xgmi-bind"          # new: keep multi-GPU pods on one xGMI hive
ANN_CU_SHARE = "amd.com/cu-share"            # new: per-pod compute-share policy (mask|temporal|hybrid)
ANN_WEBHOOK_IGNORE_LABEL = "4pd.io/webhook"  # label value "ignore" opts a pod out

# ---- node annotations (device plugin → scheduler) ------------------------------------
NODE_HANDSHAKE = "4pd.io/node-handshake-amd"
NODE_REGISTER = "4pd.io/node-amd-register"
NODE_LOCK = "4pd.io/mutex.lock"

# ---- pod annotations (scheduler → device plugin) ---------------------------------------
ASSIGNED_NODE = "4pd.io/vgpu-node"
ASSIGNED_TIME = "4pd.io/vgpu-time"
ASSIGNED_IDS = "4pd.io/vgpu-ids-new"
ASSIGNED_IDS_TO_ALLOCATE = "4pd.io/devices-to-allocate"
BIND_PHASE = "4pd.io/bind-phase"
BIND_TIME = "4pd.io/bind-time"

BIND_ALLOCATING = "allocating"
BIND_FAILED = "failed"
BIND_SUCCESS = "success"

# ---- handshake protocol (pkg/scheduler/scheduler.go:157-190) -------------------------
HANDSHAKE_REQUESTING = "Requesting_"
HANDSHAKE_REPORTED = "Reported "
HANDSHAKE_DELETED = "Deleted_"
HANDSHAKE_TIMEOUT_S = 60
NODE_LOCK_EXPIRE_S = 300

# Memory percentage sentinel meaning "not set" (pkg/device/nvidia/device.go:136-153).
MEM_PERCENT_UNSET = 101


@dataclass
class DeviceInfo:
    """One physical device as advertised by a node (pkg/api/device_register.go:13-22)."""
    id: str
    count: int          # vGPU slots (split count)
    devmem: int         # MiB (already multiplied by memory scaling)
    devcore: int        # percent (100 × cores scaling)
    type: str
    numa: int = 0
    health: bool = True
    # MI355X extensions (not part of the reference wire format; carried in a
    # separate annotation so the 7-field record stays reference-compatible)
    cus: int = 256
    xgmi_hive: str = ""
    index: int = 0
    resource: str = "amd.com/gpu"   # count resource it is advertised under (partition strategy)


@dataclass
class ContainerDeviceRequest:
    """Per-container, per-vendor request (pkg/util/types.go:50-58)."""
    nums: int
    type: str = VENDOR
    memreq: int = 0            # MiB
    mem_percentage: int = MEM_PERCENT_UNSET
    coresreq: int = 0
    resource: str = "amd.com/gpu"  # count resource the container asked for (amd.com/gpu-cpx ...)


@dataclass
class ContainerDevice:
    """One device assigned to a container (pkg/util/types.go:37-48)."""
    uuid: str
    type: str
    usedmem: int          # MiB
    usedcores: int        # percent
    idx: int = 0


ContainerDevices = list  # list[ContainerDevice]
PodDevices = list        # list[ContainerDevices], one entry per container


@dataclass
class DeviceUsage:
    """Scheduler's view of one device while scoring (pkg/util/types.go:67-76)."""
    id: str
    index: int
    used: int
    count: int
    usedmem: int
    totalmem: int
    usedcores: int
    totalcore: int
    type: str
    numa: int
    health: bool
    cus: int = 256
    xgmi_hive: str = ""
    pods: list = field(default_factory=list)
    resource: str = "amd.com/gpu"
