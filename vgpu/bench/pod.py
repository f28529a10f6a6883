"""One benchmark "pod": an ai-benchmark-equivalent workload running on one
(v)GPU under the enforcement library, driven by a launcher over stdin/stdout.

Protocol (one JSON object per line on stdout, prefixed):
    READY {...}   after the untimed warmup and a device synchronize
    <- "GO"       read from stdin
    DONE {...}    after exactly `steps` steps and a device synchronize
    <- "RCCL <rank> <world> <addr> <port>"   (optional, multi-GPU runs)
    RCCL {...}    cross-GPU all-reduce among one pod per GPU, under the shim
    <- "EXIT"
Optional post-timing probe (--cap-probe): allocate 1 GiB blocks until the
vGPU cap refuses, report how close to the cap that got (VRAM-cap accuracy).

Run standalone for debugging:  python -m vgpu.bench.pod --workload 1.1 --steps 5 --no-wait
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def emit(tag: str, obj: dict) -> None:
    sys.stdout.write(f"{tag} {json.dumps(obj)}\n")
    sys.stdout.flush()


def build(args):
    import torch
    from vgpu.models import WORKLOADS

    w = WORKLOADS[args.workload]
    torch.manual_seed(1234 + args.pod_index)
    torch.backends.cudnn.benchmark = args.find
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model = w.builder().to(dev)
    # VGPU_BENCH_DTYPE=fp32: the reference's precision (TF fp32 on V100) for the
    # sharing-ratio check; the hand-written kernels are bf16, so fp32 runs the
    # plain modules on MIOpen / hipBLASLt.
    fp32 = os.environ.get("VGPU_BENCH_DTYPE", "bf16").lower() in ("fp32", "float32")
    dtype = torch.float32 if fp32 else torch.bfloat16
    if w.kind == "image":
        model = model.to(memory_format=torch.channels_last)
    model = model.to(dtype)
    x = w.make_input(dev, dtype)
    if w.train:
        model.train()
        # The native SGD (vgpu.ops.optim: one launch per 48 bf16 tensors; VGG-16's
        # 138M parameters made PyTorch's update 15-22 % of its step).
        # VGPU_FUSED_SGD=torch: PyTorch's fused SGD, =0: PyTorch's foreach SGD (A/B).
        which = os.environ.get("VGPU_FUSED_SGD", "native")
        if which in ("0", "torch"):
            opt = torch.optim.SGD(model.parameters(), lr=1e-3, momentum=0.9, fused=(which == "torch") or None)
        else:
            from vgpu.ops.optim import SGD
            opt = SGD(model.parameters(), lr=1e-3, momentum=0.9)
            if which != "unfused":  # FC weights stepped inside their backward (VGPU_FUSED_SGD=unfused: A/B)
                opt.fuse_into_backward(model)
        ncls = 21 if w.name == "deeplab" else (2 if w.name == "lstm" else 1000)
        if w.name == "deeplab":
            target = torch.randint(0, ncls, (w.batch, *w.shape[1:]), device=dev)
        else:
            target = torch.randint(0, ncls, (w.batch,), device=dev)
        torch_loss = torch.nn.CrossEntropyLoss()
        from vgpu.ops.loss import cross_entropy

        def lossf(out, tgt):
            # one native pass for the loss and its gradient (vgpu.ops.loss):
            # classification logits and DeepLab's per-pixel logits alike
            return torch_loss(out.float(), tgt) if fp32 else cross_entropy(out, tgt)

        def step():
            opt.zero_grad(set_to_none=True)
            out = model(x)
            loss = lossf(out, target)
            loss.backward()
            opt.step()
            return loss

        def train_graph_body():
            # Whole-step capture (forward, backward, optimizer): the gradients
            # are allocated inside the graph's pool on capture and rewritten in
            # place on every replay (PyTorch "whole network capture").
            out = model(x)
            loss = lossf(out, target)
            loss.backward()
            opt.step()
    else:
        model.eval()
        from vgpu.models.resnet import FusedResNetV2Inference, ResNetV2
        from vgpu.models.vision import VGG16, NativeVGG16Inference
        conv = getattr(args, "conv", "native")
        if fp32:
            pass  # plain modules
        elif isinstance(model, ResNetV2) and not args.no_fused:
            model = FusedResNetV2Inference(model, conv=conv)
        elif isinstance(model, VGG16) and not args.no_fused and conv == "native":
            model = NativeVGG16Inference(model)
        elif hasattr(model, "fuse_for_inference"):
            model.fuse_for_inference()

        @torch.inference_mode()
        def step():
            return model(x)

    graph = None
    if args.graph and w.train and getattr(args, "train_graph", True):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):  # MIOpen find + momentum buffers before capture
                step()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        try:
            graph = torch.cuda.CUDAGraph()
            opt.zero_grad(set_to_none=True)
            with torch.cuda.graph(graph):
                train_graph_body()
        except Exception as e:  # an op without capture support (e.g. some RNN paths): eager
            sys.stderr.write(f"[pod {args.pod_index}] training hipGraph capture failed ({e}); eager\n")
            torch.cuda.synchronize()
            return w, step

        def replay_train():
            graph.replay()
        return w, replay_train
    if args.graph and not w.train:
        # Warm up on a side stream, then capture one step into a hipGraph:
        # replays cost one launch instead of hundreds (launch-bound at b≤50).
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                step()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        split = max(1, int(os.environ.get("VGPU_POD_SPLIT", "1")))
        if split > 1:
            return w, split_replay(model, x, split)
        try:
            graph = torch.cuda.CUDAGraph()
            with torch.inference_mode(), torch.cuda.graph(graph):
                model(x)
        except Exception as e:  # e.g. an op without capture support: run eagerly
            sys.stderr.write(f"[pod {args.pod_index}] hipGraph capture failed ({e}); running eagerly\n")
            torch.cuda.synchronize()
            return w, step

        def replay():
            graph.replay()
        return w, replay
    return w, step


def split_replay(model, x, split: int):
    """The batch as `split` micro-batches, one hipGraph each, replayed on their
    own streams so the kernels of different micro-batches can co-reside on the
    pod's CUs (fills tile-quantisation tails, hides per-kernel latency).  Same
    work per step; VGPU_POD_SPLIT selects it (A/B knob)."""
    import torch
    cur = torch.cuda.current_stream()
    chunks = x.chunk(split)
    streams = [torch.cuda.Stream() for _ in chunks]
    with torch.inference_mode():
        for st, xc in zip(streams, chunks):  # warm the micro-batch shape eagerly
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                model(xc)
    torch.cuda.synchronize()
    graphs = []
    for st, xc in zip(streams, chunks):
        g = torch.cuda.CUDAGraph()
        with torch.inference_mode(), torch.cuda.graph(g, stream=st):
            model(xc)
        graphs.append(g)
    torch.cuda.synchronize()

    def replay():
        cur = torch.cuda.current_stream()
        for st, g in zip(streams, graphs):
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                g.replay()
        for st in streams:
            cur.wait_stream(st)
    return replay


_PHASES = {-1: None, 0: "temporal", 1: "exploring", 2: "exploring", 3: "spatial", 4: "exploring"}


def share_state(dev: int = 0) -> dict | None:
    """The enforcement library's compute-share state in this process
    (limiter.cpp limiter_share_state): the auto policy's phase and whether it
    has decided for the current busy-member count, this pod's CUs and its
    limiter wait.  None when the library is not loaded."""
    import ctypes
    try:
        fn = ctypes.CDLL(None).vgpu_self_share_state
    except (OSError, AttributeError):
        return None
    out = (ctypes.c_int64 * 8)()
    fn(ctypes.c_int(dev), out)
    phase = _PHASES.get(int(out[0]), "exploring")
    src = ctypes.c_int(0)
    try:
        host_pid = int(ctypes.CDLL(None).vgpu_self_host_pid(ctypes.byref(src)))
    except (OSError, AttributeError):
        host_pid = 0
    return {"policy": "spatial" if out[3] else phase, "auto_phase": phase, "members": int(out[1]),
            "decided": bool(out[2]) and phase in ("temporal", "spatial"), "own_cus": bool(out[3]),
            "cus": int(out[4]), "limiter_active": bool(out[5]), "limiter_wait_ms": round(out[6] / 1e6, 3),
            # the KFD cu_occupancy cross-check: what it charged beyond the markers,
            # and how the host pid it needs was found (0 = unresolved)
            "occ_charged_ms": round(out[7] / 1e6, 3), "host_pid_src": int(src.value) if host_pid > 0 else 0}


def cap_probe() -> dict:
    import torch
    free, total = torch.cuda.mem_get_info()
    torch.cuda.empty_cache()
    blocks = []
    gib = 1 << 30
    try:
        while True:
            blocks.append(torch.empty(gib, dtype=torch.uint8, device="cuda"))
    except torch.OutOfMemoryError:
        pass
    allocated_probe = len(blocks) * gib
    reserved = torch.cuda.memory_reserved()
    del blocks
    torch.cuda.empty_cache()
    return {"mem_total_reported": total, "probe_bytes": allocated_probe,
            "reserved_at_oom": reserved}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="1.1")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--pod-index", type=int, default=0)
    ap.add_argument("--graph", action="store_true")
    ap.add_argument("--no-train-graph", dest="train_graph", action="store_false",
                    help="run training steps eagerly even with --graph")
    ap.add_argument("--find", action="store_true", help="cudnn.benchmark (MIOpen find) in warmup")
    ap.add_argument("--cap-probe", action="store_true")
    ap.add_argument("--no-fused", action="store_true", help="plain PyTorch epilogues (no HIP fusion)")
    ap.add_argument("--conv", choices=("native", "miopen"), default="native",
                    help="ResNet convolutions: fused MFMA kernels (native) or MIOpen + fused epilogues")
    ap.add_argument("--no-wait", action="store_true", help="do not wait for GO on stdin")
    ap.add_argument("--warmup-seconds", type=float, default=0.0,
                    help="keep warming up until this long has passed (lets the adaptive share policy settle)")
    ap.add_argument("--seconds", type=float, default=0.0,
                    help="run steps for this long instead of exactly --steps (share measurements)")
    ap.add_argument("--decide-timeout", type=float, default=0.0,
                    help="under the adaptive share policy, keep warming up (untimed) until the GPU's "
                         "pods have decided between time sharing and CUs of their own, at most this long")
    ap.add_argument("--share-members", type=int, default=1,
                    help="pods that share this GPU and run at once (the decision --decide-timeout waits for)")
    args = ap.parse_args(argv)

    import torch
    t_init = time.time()
    cpu = os.environ.get("VGPU_BENCH_CPU") == "1"
    if cpu:
        # orchestration rehearsal on a CPU-only host (tests): same protocol, tiny work
        from types import SimpleNamespace
        w = SimpleNamespace(batch=4)
        a = torch.randn(256, 256)

        def step():
            return a @ a

        def sync():
            pass
    else:
        w, step = build(args)
        sync = torch.cuda.synchronize
    t_w = time.monotonic()
    for _ in range(args.warmup):
        step()
    while time.monotonic() - t_w < args.warmup_seconds:
        step()
        sync()
    sync()
    # The adaptive policy (VGPU_CU_SHARE=auto) A/Bs time sharing against CU
    # claims over ~5 s of the pods' own work (limiter.cpp auto_step); a timed
    # window that starts before the decision measures the A/B, not the policy.
    decide = {"waited_s": 0.0}
    if not cpu and args.decide_timeout > 0 and os.environ.get("VGPU_CU_SHARE", "") == "auto":
        t_d = time.monotonic()
        while time.monotonic() - t_d < args.decide_timeout:
            st = share_state()
            if st is None or not st["limiter_active"] and not st["own_cus"] and st["auto_phase"] is None:
                break  # not an auto member (whole GPU, or no library)
            if st["members"] == args.share_members and (st["decided"] or args.share_members < 2):
                break  # decided for all of this GPU's pods busy at once (a lone pod has nothing to decide)
            for _ in range(4):
                step()
            sync()
        decide["waited_s"] = round(time.monotonic() - t_d, 2)
        decide["state"] = share_state()
    if cpu:
        emit("READY", {"pod": args.pod_index, "init_s": time.time() - t_init, "pid": os.getpid()})
    else:
        free, total = torch.cuda.mem_get_info()
        props = torch.cuda.get_device_properties(0)
        emit("READY", {"pod": args.pod_index, "init_s": time.time() - t_init, "mem_free": free,
                       "mem_total": total, "prop_total": props.total_memory,
                       "cus": props.multi_processor_count, "pid": os.getpid(),
                       "allocated": torch.cuda.memory_allocated(), "decide": decide})
    if not args.no_wait:
        line = sys.stdin.readline()
        if line.strip() != "GO":
            return 3
    sync()
    t0 = time.monotonic()
    steps = args.steps
    if args.seconds > 0:  # a fixed window: every pod of a share test runs the whole time
        steps = 0
        while time.monotonic() - t0 < args.seconds:
            step()
            steps += 1
            if steps % 8 == 0:
                sync()  # keep the host within a few steps of the GPU
    else:
        for _ in range(steps):
            step()
    sync()
    t1 = time.monotonic()
    res = {"pod": args.pod_index, "t0": t0, "t1": t1, "steps": steps,
           "samples": steps * w.batch, "ms_per_step": 1e3 * (t1 - t0) / max(steps, 1),
           "throughput": steps * w.batch / max(t1 - t0, 1e-9)}
    if not cpu:
        res["share"] = share_state()  # the policy the timed window ran under
    if args.cap_probe and not cpu:
        res.update(cap_probe())
    emit("DONE", res)
    if args.no_wait:
        return 0
    for line in sys.stdin:  # post-timing commands from the launcher
        cmd = line.split()
        if cmd and cmd[0] == "RCCL" and len(cmd) == 5:
            emit("RCCL", rccl_check(int(cmd[1]), int(cmd[2]), cmd[3], int(cmd[4]), cpu))
        else:
            break
    return 0


def rccl_check(rank: int, world: int, addr: str, port: int, cpu: bool, mib: int = 64, iters: int = 10) -> dict:
    """The multi-GPU data plane under the enforcement library: one pod per GPU
    forms a process group over RCCL (RCCL kernels are exempt from the shim's
    limiter) and all-reduces a `mib` MiB buffer.  Checks the sum, reports bus
    bandwidth and the transport RCCL chose per peer (NCCL_DEBUG=INFO): a pod
    sees only its own GPU, so expect SHM, not P2P/xGMI (that path is
    bench.py --pod-gpus).  Not part of the timed window."""
    import datetime

    import torch
    import torch.distributed as dist
    out = {"rank": rank, "world": world, "backend": "gloo" if cpu else "nccl"}
    dbg = f"/tmp/vgpu-rccl-{os.getpid()}.log"
    if not cpu:
        os.environ.setdefault("NCCL_DEBUG", "INFO")
        os.environ.setdefault("NCCL_DEBUG_SUBSYS", "INIT,GRAPH")
        os.environ["NCCL_DEBUG_FILE"] = dbg
    t0 = time.time()
    try:
        dev = torch.device("cpu") if cpu else torch.device("cuda", 0)
        kw = {} if cpu else {"device_id": dev}
        dist.init_process_group(out["backend"], init_method=f"tcp://{addr}:{port}", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=120), **kw)
        out["init_s"] = round(time.time() - t0, 2)
        n = (mib << 20) // 4
        y = torch.full((n,), float(rank + 1), device=dev)
        dist.all_reduce(y)
        want = world * (world + 1) / 2
        out["sum_ok"] = bool(torch.all(y == want).item())
        x = torch.ones(n, device=dev)
        for _ in range(3):
            dist.all_reduce(x)
        if not cpu:
            torch.cuda.synchronize()
        t1 = time.time()
        for _ in range(iters):
            dist.all_reduce(x)
        if not cpu:
            torch.cuda.synchronize()
        dt = (time.time() - t1) / iters
        out["ms_per_allreduce"] = round(1e3 * dt, 3)
        out["busbw_GBps"] = round(2 * (world - 1) / world * n * 4 / dt / 1e9, 1)
        dist.destroy_process_group()
        if not cpu and os.path.exists(dbg):
            sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[2]))
            from bench import rccl_transports
            out["transport"] = rccl_transports(open(dbg, errors="replace").read())
    except Exception as e:  # reported, never fatal for the benchmark
        out["error"] = f"{type(e).__name__}: {e}"[:500]
    return out


if __name__ == "__main__":
    sys.exit(main())
