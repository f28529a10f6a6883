"""Typed configuration shared by the extender, device plugin and monitor.

Reference knobs: pkg/scheduler/config/config.go:19-24 (HttpBind,
SchedulerName, DefaultMem, DefaultCores), pkg/util/types.go:85-117
(DeviceSplitCount, DeviceMemoryScaling, DeviceCoresScaling, DisableCoreLimit,
per-node DevicePluginConfigs JSON), cmd/device-plugin/nvidia/vgpucfg.go:15-133
(flags + /config/config.json per-node overrides), docs/config.md:1-45.

Precedence (lowest → highest): defaults, environment (VGPU_*), CLI flags,
per-node JSON override (device plugin only).
"""
from __future__ import annotations

import argparse
import json
import os
from dataclasses import asdict, dataclass, field, fields


@dataclass
class SchedulerConfig:
    http_bind: str = "127.0.0.1:8080"
    cert_file: str = ""
    key_file: str = ""
    scheduler_name: str = "vgpu-scheduler"
    default_mem: int = 0          # MiB; 0 → 100% of the device when nothing is requested
    default_cores: int = 0        # percent
    metrics_bind: str = ":9395"
    node_scheduler_policy: str = "binpack"   # binpack | spread (across nodes)
    gpu_scheduler_policy: str = "spread"     # spread | binpack (across devices of a node)
    xgmi_weight: float = 1.0                 # weight of the xGMI-locality term for multi-GPU pods
    register_interval_s: float = 15.0
    handshake_timeout_s: float = 60.0


@dataclass
class NodeOverride:
    name: str = ""
    devicesplitcount: int | None = None
    devicememoryscaling: float | None = None
    devicecorescaling: float | None = None


@dataclass
class DevicePluginConfig:
    node_name: str = ""
    resource_name: str = "amd.com/gpu"
    device_split_count: int = 10          # chart default (values.yaml:89-94); CLI default 2 in the reference
    device_memory_scaling: float = 1.0    # >1 enables virtual device memory (oversubscription)
    # With device_memory_scaling > 1, each container's physical HBM budget is its
    # cap / scaling (VGPU_DEVICE_MEMORY_PHYSICAL_<i>): co-located pods split the
    # HBM in proportion to their caps and page the rest (native/shim/vmem.cpp).
    vmem_physical_budget: bool = True
    device_cores_scaling: float = 1.0
    disable_core_limit: bool = False
    hw_queues_per_vgpu: int = 1           # GPU_MAX_HW_QUEUES for fractional vGPUs (0 = runtime default)
    hsa_tools_intercept: bool = False     # also hand the shim ROCr's API table (HSA_TOOLS_LIB)
    # Suspend that frees HBM on any node (VGPU_SUSPEND_EVICT): device allocations of
    # >= 32 MiB become managed ranges the shim can move to host memory, so a pod the
    # monitor suspends for a higher-priority one (SIGUSR2) gives its HBM back, and
    # gets it again when resumed (native/shim/vmem.cpp, vgpu/monitor/feedback.py).
    suspend_evict: bool = False
    partition_mode: str = ""             # SPX|DPX|QPX|CPX expected compute partition ("" = as found)
    # MIG-strategy analogue (vgpu/deviceplugin/partitions.py): none | single | mixed
    partition_strategy: str = "single"
    partition_memory: str = "split"       # split: NPS domain memory / partitions sharing it | reported
    # How a fractional vGPU's compute share is enforced (vgpu/deviceplugin/custate.py):
    #   auto      (default) pool members that measure, per GPU, time sharing against
    #             CUs of their own (share-board A/B) and keep the faster: >= 0.98 x
    #             exclusive on all 10 ai-benchmark tests at 4 x 25 % (docs/benchmarks.md)
    #   temporal  no per-container mask: the shim's GPU-time limiter with
    #             work-conserving fair-share charging (the reference's time-sliced SM limit)
    #   mask      an XCD-balanced CU mask per container (spatial isolation; temporal only
    #             when no granules are free)
    #   hybrid    CU masks for the first `max_mask_slots` fractional containers of a GPU, the
    #             rest share the remaining CUs (one pool mask) under the temporal limiter
    cu_share: str = "auto"
    max_mask_slots: int = 2
    # Temporal pool: at most this many pool members of one GPU run at a time,
    # taking turns of pool_quantum_ms (VGPU_POOL_CONCURRENCY; 0 = all at once).
    pool_concurrency: int = 0
    pool_quantum_ms: float = 50.0
    rocr_cu_mask: bool = True             # also hand the masks to ROCr (HSA_CU_MASK: internal queues too)
    host_lock_dir: str = "/tmp/vgpulock"  # node-wide unified lock + per-GPU share boards
    device_list_strategy: str = "envvar"  # envvar (device nodes in the response) | cdi-annotations | cdi-cri
    cdi_dir: str = "/var/run/cdi"
    config_file: str = "/config/config.json"
    socket_dir: str = "/var/lib/kubelet/device-plugins"
    host_lib_dir: str = "/usr/local/vgpu"
    register_interval_s: float = 30.0
    backend: str = "auto"                  # auto | amdsmi | sysfs | fake:<json>
    overrides: list = field(default_factory=list)

    def apply_node_overrides(self) -> None:
        """Per-node JSON (reference vgpucfg.go:81-107): {"nodeconfig":[{"name":...}]}"""
        p = self.config_file
        if not p or not os.path.exists(p):
            return
        try:
            cfg = json.load(open(p))
        except (OSError, ValueError):
            return
        for n in cfg.get("nodeconfig", []):
            if n.get("name") != self.node_name:
                continue
            if n.get("devicesplitcount") is not None:
                self.device_split_count = int(n["devicesplitcount"])
            if n.get("devicememoryscaling") is not None:
                self.device_memory_scaling = float(n["devicememoryscaling"])
            if n.get("devicecorescaling") is not None:
                self.device_cores_scaling = float(n["devicecorescaling"])


def add_dataclass_args(ap: argparse.ArgumentParser, cls, prefix: str = "") -> None:
    """One --flag per field (dashes), defaulting to VGPU_<FIELD> env or the dataclass default."""
    inst = cls()
    for f in fields(cls):
        if f.name in ("overrides",):
            continue
        flag = "--" + prefix + f.name.replace("_", "-")
        env = os.environ.get("VGPU_" + f.name.upper())
        default = getattr(inst, f.name)
        typ = type(default) if default is not None else str
        if typ is bool:
            dv = default if env is None else env.lower() in ("1", "true", "yes", "on")
            ap.add_argument(flag, dest=f.name, type=lambda s: s.lower() in ("1", "true", "yes", "on"),
                            default=dv, nargs="?", const=True)
        else:
            dv = default if env is None else typ(env)
            ap.add_argument(flag, dest=f.name, type=typ, default=dv)


def from_namespace(cls, ns: argparse.Namespace):
    kw = {f.name: getattr(ns, f.name) for f in fields(cls) if hasattr(ns, f.name)}
    return cls(**kw)


# Process-global scheduler config (the reference keeps package-level globals).
SCHEDULER = SchedulerConfig()


def to_dict(cfg) -> dict:
    return asdict(cfg)
