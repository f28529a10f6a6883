"""Admit benchmark pods through the real control plane.

Every pod goes through the same path as in a cluster:
* the mutating webhook;
* the scheduler extender (`Scheduler.filter` + `bind`: scoring, node lock,
  annotations);
* the device plugin's `allocate` (compute-share policy, CU masks, HBM caps, env
  contract, mounts).

The API server is the in-process fake. The node is this machine, with the one
physical GPU the pods share. The returned environments are what kubelet would
hand the containers. Container mount paths are rewritten to the host paths
behind them, so the pod processes run on the host.

Reference flow: pkg/scheduler/scheduler.go:312-402 (Filter/Bind),
pkg/device-plugin/nvidiadevice/nvinternal/plugin/server.go:280-403 (Allocate).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from pathlib import Path

from vgpu import config
from vgpu.api import resources as R
from vgpu.config import DevicePluginConfig, SchedulerConfig
from vgpu.device.base import init_default_devices
from vgpu.deviceplugin.allocate import ContainerGrant, allocate
from vgpu.deviceplugin.custate import CUMaskState
from vgpu.deviceplugin.discovery import Device
from vgpu.deviceplugin.register import register_once
from vgpu.k8s.client import KubeClient
from vgpu.k8s.fakeapi import FakeApiServer
from vgpu.scheduler.core import Scheduler
from vgpu.scheduler.webhook import handle_admission

NODE = "bench-node"


@dataclass
class AdmittedPod:
    name: str
    env: dict = field(default_factory=dict)       # container env, host paths
    grant: ContainerGrant | None = None
    cu_mask_bits: int = 0
    share: str = "none"                           # mask | temporal | none


def _pod(name: str, mem_mib: int, cores: int, priority: int | None, cu_share: str | None = None,
         count: int = 1) -> dict:
    lim = {R.RESOURCE_COUNT: str(count)}
    if mem_mib:
        lim[R.RESOURCE_MEM] = str(mem_mib)
    if cores:
        lim[R.RESOURCE_CORES] = str(cores)
    if priority is not None:
        lim[R.RESOURCE_PRIORITY] = str(priority)
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": name, "namespace": "bench", "uid": f"uid-{name}",
                         "annotations": {R.ANN_CU_SHARE: cu_share} if cu_share else {}},
            "spec": {"containers": [{"name": "main", "image": "bench", "resources": {"limits": lim}}]}}


def _host_path(value: str, mounts: list) -> str:
    for cpath, hpath, _ in sorted(mounts, key=lambda m: -len(m[0])):
        if value == cpath or value.startswith(cpath.rstrip("/") + "/"):
            return hpath + value[len(cpath):]
    return value


def admit_pods(specs: list, device_index: int, workdir: str, *, policy: str = "temporal",
               max_mask_slots: int = 2, memory_scaling: float = 1.0,
               device: Device | None = None, pool_concurrency: int = 0,
               suspend_evict: bool = False) -> list[AdmittedPod]:
    """Admit `specs` (vgpu.bench.launch.PodSpec) onto one physical GPU."""
    init_default_devices()
    config.SCHEDULER = SchedulerConfig(gpu_scheduler_policy="binpack")
    work = Path(workdir)
    host_lib = work / "host"
    lock = work / "vgpulock"
    lock.mkdir(parents=True, exist_ok=True)
    cfg = DevicePluginConfig(node_name=NODE, device_split_count=max(10, len(specs)), config_file="",
                             host_lib_dir=str(host_lib), host_lock_dir=str(lock), cu_share=policy,
                             max_mask_slots=max_mask_slots, device_memory_scaling=memory_scaling,
                             pool_concurrency=pool_concurrency, suspend_evict=suspend_evict,
                             # A/B of the ROCr tools-lib intercept (scripts/bench_ab.py tools-lib)
                             hsa_tools_intercept=os.environ.get("VGPU_HSA_TOOLS_INTERCEPT", "") in ("1", "true"))
    dev = device or Device(uuid=f"GPU-bench-{device_index}", index=device_index,
                           render_minor=128 + device_index, card=device_index)
    srv = FakeApiServer()
    url = srv.start()
    try:
        client = KubeClient(url)
        srv.add_node(NODE)
        register_once(client, NODE, [dev], cfg)
        sched = Scheduler(client)
        sched.register_from_node_annotations_once()
        cu_state = CUMaskState(str(host_lib / "containers"), policy=policy, max_mask_slots=max_mask_slots)
        out = []
        for i, sp in enumerate(specs):
            name = f"pod{i}"
            pod = _pod(name, sp.mem_mib, sp.cores, sp.priority, getattr(sp, "cu_share", None))
            review = handle_admission({"request": {"uid": name, "object": pod}})
            if not review["response"]["allowed"]:
                raise RuntimeError(f"webhook refused {name}: {review}")
            srv.add_pod(pod)
            r = sched.filter({"pod": client.get_pod("bench", name), "nodenames": [NODE]})
            if r.get("nodenames") != [NODE]:
                raise RuntimeError(f"scheduler could not place {name}: {r}")
            b = sched.bind({"podName": name, "podNamespace": "bench", "podUID": f"uid-{name}", "node": NODE})
            if b.get("error"):
                raise RuntimeError(f"bind {name}: {b['error']}")
            grant = allocate(client, cfg, R.VENDOR, [[f"{dev.uuid}-{i}"]], {dev.uuid: dev}, cu_state, NODE)[0]
            env = {k: _host_path(v, grant.mounts) for k, v in grant.envs.items()}
            env["VGPU_LOCK_DIR"] = str(lock)
            # the per-container cache dir is a host directory the plugin mounts
            region = Path(env.get("VGPU_SHARED_REGION", str(work / name / "vgpu.cache")))
            region.parent.mkdir(parents=True, exist_ok=True)
            mask = env.get("VGPU_CU_MASK_0", "0x0")
            share = env["VGPU_CU_SHARE"] if env.get("VGPU_CU_SHARE") in ("temporal", "auto") else (
                "mask" if int(mask, 16) else "none")
            out.append(AdmittedPod(name, env, grant, bin(int(mask, 16)).count("1"), share))
        return out
    finally:
        srv.stop()


def admit_multi_gpu_pod(device_indices: list[int], workdir: str, *, mem_mib: int = 0, cores: int = 0,
                        policy: str = "auto", suspend_evict: bool = False) -> AdmittedPod:
    """Admit ONE pod that asks for `len(device_indices)` vGPUs (amd.com/gpu: N)
    on a node whose devices are those physical GPUs: webhook, scheduler
    filter/bind (one device per requested vGPU), Allocate.  The returned env
    holds one cap / compute share / uuid per device (VGPU_*_<i>, i = the
    device's position inside the container) and one shared region."""
    init_default_devices()
    config.SCHEDULER = SchedulerConfig(gpu_scheduler_policy="binpack")
    work = Path(workdir)
    host_lib = work / "host"
    lock = work / "vgpulock"
    lock.mkdir(parents=True, exist_ok=True)
    n = len(device_indices)
    cfg = DevicePluginConfig(node_name=NODE, device_split_count=10, config_file="", host_lib_dir=str(host_lib),
                             host_lock_dir=str(lock), cu_share=policy, suspend_evict=suspend_evict)
    devs = [Device(uuid=f"GPU-bench-{d}", index=d, render_minor=128 + d, card=d, numa=0, xgmi_hive=0x1111)
            for d in device_indices]
    srv = FakeApiServer()
    url = srv.start()
    try:
        client = KubeClient(url)
        srv.add_node(NODE)
        register_once(client, NODE, devs, cfg)
        sched = Scheduler(client)
        sched.register_from_node_annotations_once()
        cu_state = CUMaskState(str(host_lib / "containers"), policy=policy)
        name = "ddp"
        pod = _pod(name, mem_mib, cores, None, count=n)
        review = handle_admission({"request": {"uid": name, "object": pod}})
        if not review["response"]["allowed"]:
            raise RuntimeError(f"webhook refused {name}: {review}")
        srv.add_pod(pod)
        r = sched.filter({"pod": client.get_pod("bench", name), "nodenames": [NODE]})
        if r.get("nodenames") != [NODE]:
            raise RuntimeError(f"scheduler could not place the {n}-GPU pod: {r}")
        b = sched.bind({"podName": name, "podNamespace": "bench", "podUID": f"uid-{name}", "node": NODE})
        if b.get("error"):
            raise RuntimeError(f"bind {name}: {b['error']}")
        ids = [f"{d.uuid}-0" for d in devs]
        grant = allocate(client, cfg, R.VENDOR, [ids], {d.uuid: d for d in devs}, cu_state, NODE)[0]
        env = {k: _host_path(v, grant.mounts) for k, v in grant.envs.items()}
        env["VGPU_LOCK_DIR"] = str(lock)
        region = Path(env.get("VGPU_SHARED_REGION", str(work / name / "vgpu.cache")))
        region.parent.mkdir(parents=True, exist_ok=True)
        share = env.get("VGPU_CU_SHARE", "none")
        return AdmittedPod(name, env, grant, 0, share)
    finally:
        srv.stop()


def container_visible_env(device_index: int) -> dict:
    """Device selection for a host process standing in for the container (the
    container would only see its own render node)."""
    return {"HIP_VISIBLE_DEVICES": str(device_index), "ROCR_VISIBLE_DEVICES": None}


def apply_env(base: dict, env: dict) -> dict:
    out = dict(base)
    for k, v in env.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = v
    return out


__all__ = ["admit_pods", "admit_multi_gpu_pod", "AdmittedPod", "apply_env", "container_visible_env", "NODE"]

if __name__ == "__main__":  # pragma: no cover - manual inspection
    import json
    import tempfile
    from vgpu.bench.launch import PodSpec
    pods = admit_pods([PodSpec(cores=25, mem_mib=72000)] * 4, 0, tempfile.mkdtemp())
    print(json.dumps([{"name": p.name, "share": p.share, "cus": p.cu_mask_bits,
                       "env": {k: v for k, v in p.env.items() if k.startswith(("VGPU", "GPU"))}}
                      for p in pods], indent=1), flush=True)
    os._exit(0)
