"""The device plugin's Allocate: turn the scheduler's pod annotations into the
container runtime configuration for one MI355X vGPU container.

Reference: pkg/device-plugin/nvidiadevice/nvinternal/plugin/server.go:280-403
(find pending pod, pop the next container's device list, check the count,
envs CUDA_DEVICE_MEMORY_LIMIT_<i>/SM_LIMIT/SHARED_CACHE/OVERSUBSCRIBE, mounts
libvgpu.so + per-container cache dir + /tmp/vgpulock + /etc/ld.so.preload
unless CUDA_DISABLE_CONTROL), pkg/util/util.go:174-236 (GetNextDeviceRequest,
EraseNextDeviceTypeFromAnnotation), pkg/device/devices.go:54-91
(PodAllocationTrySuccess / Success / Failed); Hygon variant
pkg/device-plugin/hygon/dcu/server.go:461-546 (/dev/kfd + /dev/dri nodes,
CU mask per container).

MI355X specifics: /dev/kfd + /dev/dri/renderD<minor> (+ card) per device;
limits are per device (`VGPU_DEVICE_CU_LIMIT_<i>`), an XCD-balanced CU mask per
fractional device, a HW-queue budget for fractional vGPUs, and ordinal i in
the container = i-th assigned device in physical (KFD) order, which is how
ROCr enumerates the render nodes the container can open.
"""
from __future__ import annotations

import logging
import time
from dataclasses import dataclass, field

from vgpu.api import resources as R
from vgpu.api.codec import decode_pod_devices, encode_pod_devices
from vgpu.api.env import (ENV_CU_LIMIT, ENV_CU_MASK, ENV_CU_SHARE, ENV_CORE_POLICY, ENV_DISABLE_CONTROL, ENV_MEM_LIMIT,
                          ENV_BDF, ENV_MEM_PHYSICAL, ENV_OVERSUBSCRIBE, ENV_SHARED_REGION, ENV_SUSPEND_EVICT, ENV_UUID, PRELOAD_FILE,
                          SHIM_NAME,
                          format_mask)
from vgpu.api.resources import ContainerDevice
from vgpu.config import DevicePluginConfig
from vgpu.k8s import objects as O
from vgpu.k8s.client import ApiError, KubeClient
from vgpu.k8s.nodelock import release_node_lock

from vgpu.device.cualloc import CULayout

from .cdi import device_names as cdi_device_names
from .custate import POLICIES, CUMaskState
from .discovery import Device

log = logging.getLogger("vgpu.deviceplugin.allocate")

CONTAINER_LIB_DIR = "/usr/local/vgpu"
CONTAINER_CACHE_DIR = "/var/run/vgpu"
CONTAINER_LOCK_DIR = "/tmp/vgpulock"


class AllocateError(Exception):
    pass


@dataclass
class ContainerGrant:
    envs: dict = field(default_factory=dict)
    mounts: list = field(default_factory=list)     # (container_path, host_path, read_only)
    devices: list = field(default_factory=list)    # (container_path, host_path, permissions)
    annotations: dict = field(default_factory=dict)
    cdi_devices: list = field(default_factory=list)  # fully-qualified CDI names (cdi-cri strategy)


CDI_ANNOTATION = "cdi.k8s.io/amd-vgpu"


def get_pending_pod(client: KubeClient, node: str) -> dict | None:
    """The pod being allocated on this node: bound here, bind-phase allocating,
    oldest bind-time first (only one should exist: the node lock serialises).
    Uses a spec.nodeName field selector instead of listing every pod in the
    cluster (reference util.go:41-66)."""
    pods = client.list_pods(field_selector=f"spec.nodeName={node}")
    cands = []
    for p in pods:
        a = O.annotations(p)
        if a.get(R.BIND_PHASE) != R.BIND_ALLOCATING:
            continue
        if a.get(R.ASSIGNED_NODE, node) != node:
            continue
        cands.append((int(a.get(R.BIND_TIME, "0") or 0), p))
    if not cands:
        return None
    cands.sort(key=lambda t: t[0])
    return cands[0][1]


def next_device_request(vendor: str, pod: dict) -> tuple[int, list[ContainerDevice]]:
    pd = decode_pod_devices(O.annotations(pod).get(R.ASSIGNED_IDS_TO_ALLOCATE, ""))
    for i, ctr in enumerate(pd):
        devs = [d for d in ctr if d.type == vendor]
        if devs:
            return i, devs
    raise AllocateError("device request not found")


def erase_next_device_type(client: KubeClient, vendor: str, pod: dict) -> dict:
    a = O.annotations(pod)
    pd = decode_pod_devices(a.get(R.ASSIGNED_IDS_TO_ALLOCATE, ""))
    for i, ctr in enumerate(pd):
        if any(d.type == vendor for d in ctr):
            pd[i] = [d for d in ctr if d.type != vendor]
            break
    enc = encode_pod_devices(pd)
    pod["metadata"]["annotations"][R.ASSIGNED_IDS_TO_ALLOCATE] = enc
    client.patch_pod_annotations(O.namespace(pod), O.name(pod), {R.ASSIGNED_IDS_TO_ALLOCATE: enc})
    return pod


def allocation_try_success(client: KubeClient, node: str, pod: dict) -> None:
    """Success once no device of any vendor remains to allocate."""
    p = client.get_pod(O.namespace(pod), O.name(pod))
    left = decode_pod_devices(O.annotations(p).get(R.ASSIGNED_IDS_TO_ALLOCATE, ""))
    if any(ctr for ctr in left):
        return
    client.patch_pod_annotations(O.namespace(p), O.name(p), {R.BIND_PHASE: R.BIND_SUCCESS})
    try:
        release_node_lock(client, node)
    except Exception as e:  # lock expiry covers us
        log.warning("release node lock %s: %s", node, e)


def allocation_failed(client: KubeClient, node: str, pod: dict | None) -> None:
    if pod is not None:
        try:
            client.patch_pod_annotations(O.namespace(pod), O.name(pod), {R.BIND_PHASE: R.BIND_FAILED})
        except ApiError as e:
            log.error("mark pod failed: %s", e)
    try:
        release_node_lock(client, node)
    except Exception as e:
        log.warning("release node lock %s: %s", node, e)


def _ctr_env_names(pod: dict, idx: int) -> set[str]:
    ctrs = O.containers(pod)
    if idx >= len(ctrs):
        return set()
    return {e.get("name") for e in ctrs[idx].get("env") or []}


def mask_ranges(mask: int) -> str:
    """CU bit set → ROCr HSA_CU_MASK list syntax, e.g. 0b1110011 → '0-1,4-6'."""
    out, bit = [], 0
    while mask >> bit:
        if mask >> bit & 1:
            start = bit
            while mask >> (bit + 1) & 1:
                bit += 1
            out.append(str(start) if start == bit else f"{start}-{bit}")
        bit += 1
    return ",".join(out)


def build_container_grant(cfg: DevicePluginConfig, pod: dict, ctr_idx: int, devreq: list[ContainerDevice],
                          devices: dict[str, Device], cu_state: CUMaskState) -> ContainerGrant:
    ctrs = O.containers(pod)
    ctr_name = ctrs[ctr_idx].get("name", str(ctr_idx)) if ctr_idx < len(ctrs) else str(ctr_idx)
    key = f"{O.uid(pod)}_{ctr_name}"
    ordered = sorted(devreq, key=lambda d: devices[d.uuid].index if d.uuid in devices else 1 << 30)
    for d in ordered:
        if d.uuid not in devices:
            raise AllocateError(f"unknown device {d.uuid}")
    layouts = {d.uuid: CULayout(total_cus=devices[d.uuid].cus or 256,
                                num_xcc=max(devices[d.uuid].num_xcc or 1, 1)) for d in ordered}
    pod_policy = O.annotations(pod).get(R.ANN_CU_SHARE)
    if pod_policy is not None and pod_policy not in POLICIES:
        log.warning("pod %s: ignoring %s=%r (not one of %s)", O.name(pod), R.ANN_CU_SHARE, pod_policy, POLICIES)
        pod_policy = None
    shares = {} if cfg.disable_core_limit else cu_state.allocate(
        key, [(d.uuid, d.usedcores) for d in ordered], layouts, policy=pod_policy)
    g = ContainerGrant()
    env_names = _ctr_env_names(pod, ctr_idx)
    fractional = False
    temporal = False
    rocr_masks: list[str] = []
    for i, d in enumerate(ordered):
        dev = devices[d.uuid]
        g.envs[ENV_MEM_LIMIT.format(i=i)] = f"{d.usedmem}m"
        if cfg.device_memory_scaling > 1 and cfg.vmem_physical_budget and d.usedmem > 0:
            g.envs[ENV_MEM_PHYSICAL.format(i=i)] = f"{int(d.usedmem / cfg.device_memory_scaling)}m"
        g.envs[ENV_UUID.format(i=i)] = d.uuid
        if dev.bdf:
            # amd-smi / rocm-smi inside the pod enumerate every GPU of the node
            # (sysfs is not namespaced): the shim keeps and orders the ones
            # whose PCI address is the container's (hooks_smi.cpp).
            g.envs[ENV_BDF.format(i=i)] = dev.bdf
        if 0 < d.usedcores < 100 and not cfg.disable_core_limit:
            fractional = True
            g.envs[ENV_CU_LIMIT.format(i=i)] = str(d.usedcores)
            sg = shares.get(d.uuid)
            if sg and sg.mask:
                g.envs[ENV_CU_MASK.format(i=i)] = format_mask(sg.mask)
                rocr_masks.append(f"{i}:{mask_ranges(sg.mask)}")
            temporal |= bool(sg and sg.temporal)
        g.devices.append((f"/dev/dri/renderD{dev.render_minor}", f"/dev/dri/renderD{dev.render_minor}", "rw"))
        g.devices.append((f"/dev/dri/card{dev.card}", f"/dev/dri/card{dev.card}", "rw"))
    g.devices.insert(0, ("/dev/kfd", "/dev/kfd", "rw"))
    if temporal:
        # Pool member: shares the device's unmasked CUs with the other pool
        # members under the shim's GPU-time limiter (fair-share board in the
        # node-wide lock dir); no mask is derived from the limit.  Under the
        # auto policy it may later claim CUs of its own (limiter.cpp auto_step).
        g.envs[ENV_CU_SHARE] = "auto" if (pod_policy or cfg.cu_share) == "auto" else "temporal"
        g.envs["VGPU_CU_MASK_FROM_LIMIT"] = "false"
        if cfg.pool_concurrency > 0:
            g.envs["VGPU_POOL_CONCURRENCY"] = str(cfg.pool_concurrency)
            g.envs["VGPU_POOL_QUANTUM_MS"] = f"{cfg.pool_quantum_ms:g}"
    if rocr_masks and cfg.rocr_cu_mask and "HSA_CU_MASK" not in env_names:
        # ROCr applies HSA_CU_MASK to every AQL queue it creates, its internal
        # blit/utility queue included — the one queue the shim's
        # hsa_queue_create hook never sees.  Same logical CU bits as the shim's
        # hsa_amd_queue_cu_set_mask (tests/test_gpu_shim.py census).
        g.envs["HSA_CU_MASK"] = ";".join(rocr_masks)
    if fractional and cfg.hw_queues_per_vgpu and "GPU_MAX_HW_QUEUES" not in env_names:
        g.envs["GPU_MAX_HW_QUEUES"] = str(cfg.hw_queues_per_vgpu)
    g.envs[ENV_SHARED_REGION] = f"{CONTAINER_CACHE_DIR}/vgpu.cache"
    if cfg.hsa_tools_intercept and "HSA_TOOLS_LIB" not in env_names:
        # ROCr hands the shim its API table in hsa_init: queue and pool calls
        # are enforced even for code that resolved hsa_* by hand.
        g.envs["HSA_TOOLS_LIB"] = f"{CONTAINER_LIB_DIR}/{SHIM_NAME}"
    if cfg.device_memory_scaling > 1:
        g.envs[ENV_OVERSUBSCRIBE] = "true"
    if cfg.suspend_evict:
        g.envs[ENV_SUSPEND_EVICT] = "true"
    if cfg.disable_core_limit:
        g.envs[ENV_CORE_POLICY] = "disable"
    host_cache = f"{cfg.host_lib_dir}/containers/{key}"
    g.mounts.append((f"{CONTAINER_LIB_DIR}/{SHIM_NAME}", f"{cfg.host_lib_dir}/{SHIM_NAME}", True))
    g.mounts.append((CONTAINER_CACHE_DIR, host_cache, False))
    g.mounts.append((CONTAINER_LOCK_DIR, cfg.host_lock_dir, False))
    if ENV_DISABLE_CONTROL not in env_names and "CUDA_DISABLE_CONTROL" not in env_names:
        g.mounts.append(("/etc/ld.so.preload", f"{cfg.host_lib_dir}/{PRELOAD_FILE}", True))
    g.annotations["amd.com/vgpu-devices"] = ",".join(d.uuid for d in ordered)
    if cfg.device_list_strategy in ("cdi-annotations", "cdi-cri"):
        # Device nodes come from the CDI spec the plugin wrote at start
        # (reference nvinternal/plugin/server.go:322-344 + cdi/cdi.go).
        g.devices = []
        names = cdi_device_names([d.uuid for d in ordered])
        if cfg.device_list_strategy == "cdi-annotations":
            g.annotations[CDI_ANNOTATION] = ",".join(names)
        else:
            g.cdi_devices = names
    return g


def allocate(client: KubeClient, cfg: DevicePluginConfig, vendor: str, requests: list[list[str]],
             devices: dict[str, Device], cu_state: CUMaskState, node: str) -> list[ContainerGrant]:
    """requests: kubelet's fake device IDs per container (only their count matters:
    the real devices come from the scheduler's annotations)."""
    pod = None
    try:
        pod = get_pending_pod(client, node)
        if pod is None:
            raise AllocateError(f"no pending pod on node {node}")
        out = []
        for ids in requests:
            idx, devreq = next_device_request(vendor, pod)
            if len(devreq) != len(ids):
                raise AllocateError("device number not matched")
            out.append(build_container_grant(cfg, pod, idx, devreq, devices, cu_state))
            pod = erase_next_device_type(client, vendor, pod)
        allocation_try_success(client, node, pod)
        return out
    except (AllocateError, ApiError) as e:
        log.error("allocate failed on %s: %s", node, e)
        allocation_failed(client, node, pod)
        raise
