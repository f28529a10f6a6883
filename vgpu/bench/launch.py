"""Node-local pod launcher: N pods sharing one physical GPU.

Pods are admitted through the real control plane (vgpu.bench.control: webhook,
scheduler filter/bind, device plugin Allocate against an in-process API
server).  Each one runs with the env Allocate returned: its own shared region,
HBM cap, compute limit, CU mask or pool membership.  LD_PRELOAD of libvgpu.so
stands in for the /etc/ld.so.preload mount.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile
import time
from dataclasses import dataclass, field
from pathlib import Path

from vgpu.api.env import DeviceGrant, container_env
from vgpu.device.cualloc import MI355X, alloc_cu_mask
from vgpu.native import preload_env, shim_path

REPO = Path(__file__).resolve().parents[2]


@dataclass
class PodSpec:
    workload: str = "1.1"
    mem_mib: int = 144000
    cores: int = 50
    priority: int | None = None
    extra_env: dict = field(default_factory=dict)
    cu_share: str | None = None   # per-pod policy override (annotation amd.com/cu-share)


def visible_device_for(local_rank: int) -> str:
    """Device id (in the parent's visible-device numbering) for one rank.
    VGPU_BENCH_DEVICES (a rank -> device list, e.g. "0,0" to put two ranks on
    one GPU in a rehearsal) takes precedence over the visible-device lists."""
    lst = (os.environ.get("VGPU_BENCH_DEVICES") or os.environ.get("HIP_VISIBLE_DEVICES")
           or os.environ.get("CUDA_VISIBLE_DEVICES"))
    if lst:
        ids = [s for s in lst.split(",") if s.strip()]
        return ids[local_rank % len(ids)].strip()
    return str(local_rank)


class Pod:
    def __init__(self, idx: int, proc: subprocess.Popen, region: str, env: dict):
        self.idx = idx
        self.proc = proc
        self.region = region
        self.env = env
        self.ready: dict | None = None
        self.done: dict | None = None
        self.mask_bits = 0  # CUs in the pod's mask (0 = no mask)
        self.share = "none"  # mask | temporal | none (how its compute share is enforced)

    def read_tagged(self, tag: str, timeout: float, progress=None) -> dict:
        """Read stdout lines until `TAG {json}`; raises on EOF or timeout."""
        import selectors
        sel = selectors.DefaultSelector()
        sel.register(self.proc.stdout, selectors.EVENT_READ)
        deadline = time.monotonic() + timeout
        last_note = time.monotonic()
        while True:
            left = deadline - time.monotonic()
            if left <= 0:
                raise TimeoutError(f"pod {self.idx}: no {tag} within {timeout:.0f}s")
            if not sel.select(timeout=min(left, 30.0)):
                if progress and time.monotonic() - last_note > 55:
                    progress(f"pod {self.idx}: waiting for {tag} ...")
                    last_note = time.monotonic()
                continue
            line = self.proc.stdout.readline()
            if not line:
                rc = self.proc.wait()
                raise RuntimeError(f"pod {self.idx} exited (rc={rc}) before {tag}")
            if line.startswith(tag + " "):
                return json.loads(line[len(tag) + 1:])
            sys.stderr.write(f"[pod{self.idx}] {line}")

    def send(self, msg: str) -> None:
        self.proc.stdin.write(msg + "\n")
        self.proc.stdin.flush()


def launch_pods(specs: list[PodSpec], device: str, *, steps: int, warmup: int, shim: bool = True,
                graph: bool = True, cap_probe: bool = False, find: bool = False,
                workdir: str | None = None, oversubscribe: bool = False,
                hw_queues: int | None = None, fused: bool = True,
                conv: str = "native", cu_share: str = "temporal", memory_scaling: float = 1.0,
                pool_concurrency: int = 0, seconds: float = 0.0, warmup_seconds: float = 0.0,
                decide_timeout: float = 0.0) -> list[Pod]:
    """Start one process per pod on physical device `device`.

    cu_share: how a fractional pod's compute share is enforced.
      hybrid, mask, temporal: the device plugin's share policy
        (vgpu/deviceplugin/custate.py).  Pods are admitted through the real
        control plane (webhook → scheduler filter/bind → device plugin
        Allocate, vgpu.bench.control) and run with exactly the env Allocate
        returns.
      group2, group2i: A/B tools outside the plugin.  Pods 2k and 2k+1
        (group2i: k and k+n/2) share one mask sized for both."""
    workdir = workdir or tempfile.mkdtemp(prefix="vgpu-pods-")
    # Node-wide lock directory shared by the pods of this node (the device
    # plugin mounts the host's /tmp/vgpulock into every vGPU container).
    lock_dir = str(Path(workdir) / "vgpulock")
    Path(lock_dir).mkdir(parents=True, exist_ok=True)
    admitted = None
    if cu_share in ("hybrid", "mask", "temporal", "auto"):
        from vgpu.bench.control import admit_pods
        admitted = admit_pods(specs, int(device) if device.isdigit() else 0, workdir, policy=cu_share,
                              memory_scaling=max(memory_scaling, 2.0 if oversubscribe else 1.0),
                              pool_concurrency=pool_concurrency)
    used = 0
    pods = []
    group_masks: dict[int, int] = {}
    for i, sp in enumerate(specs):
        mask = 0
        if admitted is not None:
            cenv = dict(admitted[i].env)
            mask_bits = admitted[i].cu_mask_bits
            if "HSA_CU_MASK" in cenv and device.isdigit():
                # In a pod ROCr enumerates only the container's GPUs (index 0 here);
                # a bench pod sees the whole node, so name the physical ordinal.
                cenv["HSA_CU_MASK"] = ";".join(f"{device}:{e.partition(':')[2]}"
                                               for e in cenv["HSA_CU_MASK"].split(";"))
        else:
            if sp.cores and sp.cores < 100 and cu_share in ("group2", "group2i"):
                g = i // 2 if cu_share == "group2" else i % max(1, (len(specs) + 1) // 2)
                if g not in group_masks:
                    m = alloc_cu_mask(used, min(100, 2 * sp.cores), MI355X)
                    if m is None:
                        raise RuntimeError(f"{cu_share}: no CUs left for the mask of pod group {g}")
                    group_masks[g] = m
                    used |= m
                mask = group_masks[g]
            region = str(Path(workdir) / f"pod{i}" / "vgpu.cache")
            Path(region).parent.mkdir(parents=True, exist_ok=True)
            grant = DeviceGrant(uuid=f"GPU-{device}", index=int(device) if device.isdigit() else 0,
                                mem_mib=sp.mem_mib, cores=sp.cores, cu_mask=mask)
            cenv = container_env([grant], region, priority=sp.priority, oversubscribe=oversubscribe,
                                 visible_var=ENV_PLACEHOLDER, lock_dir=lock_dir)
            cenv.pop(ENV_PLACEHOLDER, None)
            mask_bits = bin(mask).count("1")
        if sp.priority is not None:
            cenv.setdefault("VGPU_TASK_PRIORITY", str(sp.priority))
        # A pod is its own program, not a torchrun worker: drop the launcher's
        # rendezvous variables (TORCHELASTIC_USE_AGENT_STORE would make a pod's
        # own process group wait on the agent's store).
        env = {k: v for k, v in os.environ.items()
               if not k.startswith(("TORCHELASTIC_", "TORCH_ELASTIC_")) and k not in TORCHRUN_VARS}
        env["HIP_VISIBLE_DEVICES"] = device
        env.pop("CUDA_VISIBLE_DEVICES", None)
        env["PYTHONPATH"] = str(REPO) + os.pathsep + env.get("PYTHONPATH", "")
        env.setdefault("MIOPEN_LOG_LEVEL", "3")
        if hw_queues:
            # HW-queue budget of a fractional vGPU (see vgpu/deviceplugin/allocate.py)
            env["GPU_MAX_HW_QUEUES"] = str(hw_queues)
        if shim:
            env.update(cenv)
            if "HSA_TOOLS_LIB" in env:  # the container path of the library -> this host's build
                env["HSA_TOOLS_LIB"] = str(shim_path())
            env = preload_env(env)
        env.update(sp.extra_env)
        cmd = [sys.executable, "-u", "-m", "vgpu.bench.pod", "--workload", sp.workload,
               "--steps", str(steps), "--warmup", str(warmup), "--pod-index", str(i)]
        if graph:
            cmd.append("--graph")
        if cap_probe:
            cmd.append("--cap-probe")
        if find:
            cmd.append("--find")
        if not fused:
            cmd.append("--no-fused")
        cmd += ["--conv", conv]
        if seconds > 0:
            cmd += ["--seconds", str(seconds)]
        if warmup_seconds > 0:
            cmd += ["--warmup-seconds", str(warmup_seconds)]
        if decide_timeout > 0:
            cmd += ["--decide-timeout", str(decide_timeout), "--share-members", str(len(specs))]
        proc = subprocess.Popen(cmd, env=env, stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                text=True, bufsize=1, cwd=str(REPO))
        pod = Pod(i, proc, cenv.get("VGPU_SHARED_REGION", ""), {k: v for k, v in cenv.items()})
        pod.mask_bits = mask_bits
        pod.share = admitted[i].share if admitted is not None else cu_share
        pods.append(pod)
    return pods


ENV_PLACEHOLDER = "__VGPU_UNUSED_VISIBLE__"
TORCHRUN_VARS = {"RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
                 "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT"}


def shim_available() -> bool:
    return shim_path().exists()
