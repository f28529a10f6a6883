"""Environment contract between the device plugin's ``Allocate`` and the
in-container enforcement library (native/shim/region.cpp:limits_from_env).

Reference: pkg/device-plugin/nvidiadevice/nvinternal/plugin/server.go:335-396
(CUDA_DEVICE_MEMORY_LIMIT_<i>=<MiB>m, CUDA_DEVICE_SM_LIMIT,
CUDA_DEVICE_MEMORY_SHARED_CACHE, CUDA_OVERSUBSCRIBE,
GPU_CORE_UTILIZATION_POLICY, mounts of libvgpu.so / ld.so.preload /
/tmp/vgpulock), pkg/device/nvidia/device.go:49-60 (CUDA_TASK_PRIORITY).

Differences (SURVEY.md §7.5 "do not copy"): the compute limit is per device
(``VGPU_DEVICE_CU_LIMIT_<i>``) instead of one value per container, and each
device may carry an XCD-balanced CU mask (``VGPU_CU_MASK_<i>``).
"""
from __future__ import annotations

from dataclasses import dataclass

ENV_MEM_LIMIT = "VGPU_DEVICE_MEMORY_LIMIT_{i}"
ENV_CU_LIMIT = "VGPU_DEVICE_CU_LIMIT_{i}"
ENV_CU_MASK = "VGPU_CU_MASK_{i}"
# "temporal": the container's compute share is enforced in time (GPU-time limiter);
# a VGPU_CU_MASK_<i> given with it is the shared pool the container runs on.
ENV_CU_SHARE = "VGPU_CU_SHARE"
ENV_UUID = "VGPU_DEVICE_UUID_{i}"
ENV_BDF = "VGPU_DEVICE_BDF_{i}"  # PCI address of ordinal i: the shim matches smi handles by it
ENV_SHARED_REGION = "VGPU_SHARED_REGION"
ENV_OVERSUBSCRIBE = "VGPU_OVERSUBSCRIBE"
# Physical HBM budget of an oversubscribed container (MiB, "m" suffix): virtual
# device memory keeps at most this much resident (native/shim/vmem.cpp).
ENV_MEM_PHYSICAL = "VGPU_DEVICE_MEMORY_PHYSICAL_{i}"
# Opt-in: allocations >= VGPU_VMEM_MANAGED_MIN_MB are managed ranges even without
# oversubscription, so a suspended container's HBM can be evicted to host memory.
ENV_SUSPEND_EVICT = "VGPU_SUSPEND_EVICT"
ENV_PRIORITY = "VGPU_TASK_PRIORITY"
ENV_CORE_POLICY = "GPU_CORE_UTILIZATION_POLICY"
ENV_OOM_KILLER = "ACTIVE_OOM_KILLER"
ENV_DISABLE_CONTROL = "VGPU_DISABLE_CONTROL"
ENV_LOG_LEVEL = "VGPU_LOG_LEVEL"
ENV_VISIBLE = "ROCR_VISIBLE_DEVICES"
ENV_HIP_VISIBLE = "HIP_VISIBLE_DEVICES"
# Node-wide lock directory (unified lock + per-GPU share boards); defaults to
# HOST_LOCK_DIR, which Allocate mounts into the container at the same path.
ENV_LOCK_DIR = "VGPU_LOCK_DIR"

# Host paths (same layout as the reference: server.go:347,354-369)
HOST_LIB_DIR = "/usr/local/vgpu"
HOST_CONTAINERS_DIR = "/usr/local/vgpu/containers"
HOST_LOCK_DIR = "/tmp/vgpulock"
SHIM_NAME = "libvgpu.so"
PRELOAD_FILE = "ld.so.preload"


def format_mask(mask: int) -> str:
    return f"0x{mask:x}"


@dataclass
class DeviceGrant:
    """What one container gets on one physical device."""
    uuid: str
    index: int               # physical index on the node (for /dev/dri and ROCR_VISIBLE_DEVICES)
    mem_mib: int             # cap in MiB (0 = unlimited)
    cores: int               # percent (0 = unlimited / best effort)
    cu_mask: int = 0         # logical CU mask (0 = none)


def container_env(grants: list[DeviceGrant], region_path: str | None, *,
                  oversubscribe: bool = False, priority: int | None = None,
                  core_policy: str | None = None, disable_core_limit: bool = False,
                  visible_var: str = ENV_VISIBLE, lock_dir: str | None = None) -> dict[str, str]:
    """Env vars for one container. Device ordinal i inside the container is
    grants[i] (ROCm honours ROCR_VISIBLE_DEVICES natively)."""
    env: dict[str, str] = {}
    if grants:
        env[visible_var] = ",".join(str(g.index) for g in grants)
    for i, g in enumerate(grants):
        if g.mem_mib > 0:
            env[ENV_MEM_LIMIT.format(i=i)] = f"{g.mem_mib}m"
        if g.cores > 0 and not disable_core_limit:
            env[ENV_CU_LIMIT.format(i=i)] = str(min(g.cores, 100))
        if g.cu_mask and not disable_core_limit:
            env[ENV_CU_MASK.format(i=i)] = format_mask(g.cu_mask)
        env[ENV_UUID.format(i=i)] = g.uuid
    if region_path:
        env[ENV_SHARED_REGION] = region_path
    if lock_dir:
        env[ENV_LOCK_DIR] = lock_dir
    if oversubscribe:
        env[ENV_OVERSUBSCRIBE] = "true"
    if priority is not None:
        env[ENV_PRIORITY] = str(priority)
    if disable_core_limit:
        env[ENV_CORE_POLICY] = "disable"
    elif core_policy:
        env[ENV_CORE_POLICY] = core_policy
    return env
