"""Data-parallel training of the ai-benchmark training workloads, one process
per (v)GPU, gradients all-reduced over RCCL (torch.distributed backend "nccl"
is RCCL on ROCm) — the multi-GPU data-plane of SURVEY.md §2.9 ("benchmark
harness only: PyTorch DDP over RCCL/xGMI for the 1/2/4/8-GPU scaling curve;
the shim must not break RCCL").  It is also what a multi-GPU vGPU pod runs
(`bench.py --pod-gpus N`: the pod is admitted through the control plane with
`amd.com/gpu: N`, torchrun inside it starts one rank per visible device under
the enforcement library).

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        -m vgpu.parallel.ddp --workload 1.2 --steps 20 --warmup 5

Design for MI355X over xGMI (7 point-to-point links per GPU, ≈153 GB/s each):

* Gradients live in one flat buffer per dtype; every parameter's `.grad` is a
  view into it (no copy into a bucket, no copy out).  The buffer is cut into
  few, large buckets (`--bucket-mb`, default 64 MB: a ResNet-V2-50 bf16 step
  is ~50 MB of gradients, i.e. one or two ring collectives, which are per-link
  bound) in reverse parameter order — the order backward produces them.
* A post-accumulate hook counts each bucket's gradients; when a bucket is
  complete it is pre-scaled by 1/world and all-reduced asynchronously, so the
  collective runs beside the rest of the backward pass.  The optimizer waits
  for every bucket.
* The whole step — forward, backward with its collectives, fused SGD — is
  captured into one hipGraph after a warmup on a side stream and replayed
  (`--graph`, default on GPU): the same single-launch step as a single pod
  (vgpu/bench/pod.py), which a DDP step with PyTorch's reducer cannot be.
  RCCL's kernels inside the replay are RCCL's: the enforcement library exempts
  a graph with collective kernel nodes from the temporal limiter
  (native/shim/hooks_hip.cpp hipGraphLaunch).
* Replicas start identical (rank 0's weights are broadcast) and stay
  identical (averaged gradients, same optimizer).

On CPU (tests) the same code runs eagerly over gloo.  Prints one JSON line on
rank 0: aggregate images/s over all ranks (max step time over ranks).
"""
from __future__ import annotations

import argparse
import json
import os
import time


def setup(backend: str | None = None, device: str | None = None):
    """init_process_group from torchrun's env; returns (rank, world, device).

    device="cuda" with backend="gloo" keeps the model on the GPU and reduces
    over gloo: the only way to put several ranks on ONE GPU, which RCCL refuses
    ("Duplicate GPU detected", profiles/r2/rccl_two_ranks_one_gpu.log)."""
    import torch
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    use_gpu = torch.cuda.is_available() and (backend != "gloo" or device == "cuda")
    if use_gpu:
        torch.cuda.set_device(local % torch.cuda.device_count())
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")
    if not dist.is_initialized():
        be = backend or ("nccl" if use_gpu else "gloo")
        kw = {"device_id": device} if be == "nccl" else {}
        dist.init_process_group(be, rank=rank, world_size=world, **kw)
    return rank, world, device


def build_model(workload: str, device, dtype=None, shrink: bool = False):
    """The workload's training model on `device` (bf16 channels_last on GPU).
    shrink: a one-block-per-stage ResNet for CPU tests."""
    import torch
    from vgpu.models import WORKLOADS
    w = WORKLOADS[workload]
    if shrink and w.name.startswith("resnet"):
        from vgpu.models.resnet import ResNetV2
        model = ResNetV2([1, 1, 1, 1], num_classes=10)
    else:
        model = w.builder()
    model = model.to(device)
    if w.kind == "image":
        model = model.to(memory_format=torch.channels_last)
    if dtype is None:
        dtype = torch.bfloat16 if device.type == "cuda" else torch.float32
    return w, model.to(dtype).train()


class GradBuckets:
    """Flat gradient buffers, bucketed all-reduce launched from the backward.

    `begin()` zeroes the gradients (one kernel per buffer); during backward each
    complete bucket is all-reduced asynchronously; `finish()` makes the current
    stream wait for every bucket.  Usable eagerly and under graph capture."""

    def __init__(self, params, bucket_mb: int = 64, world: int | None = None, group=None):
        import torch
        import torch.distributed as dist
        self.params = [p for p in params if p.requires_grad]
        self.world = world or dist.get_world_size(group)
        self.group = group
        cap = max(1, bucket_mb) << 20
        self.flat = {}
        self.buckets = []    # [(flat view, [params])], in the order backward completes them
        self.bucket_of = {}  # id(param) -> bucket index
        by_dtype: dict = {}
        for p in self.params:
            by_dtype.setdefault(p.dtype, []).append(p)
        for dt, ps in by_dtype.items():
            n = sum(p.numel() for p in ps)
            flat = torch.zeros(n, dtype=dt, device=ps[0].device)
            self.flat[dt] = flat
            # reverse order: the last layers' gradients are ready first
            off = n
            cur, cur_bytes, hi = [], 0, n
            for p in reversed(ps):
                off -= p.numel()
                # the parameter's own (dense) strides -- channels_last conv weights
                # included: autograd accumulates in place only into a grad that
                # obeys the layout contract, and the fused optimizer needs it too
                p.grad = torch.as_strided(flat, p.size(), p.stride(), off)
                cur.append(p)
                cur_bytes += p.numel() * p.element_size()
                if cur_bytes >= cap:
                    self._add_bucket(flat[off:hi], cur)
                    cur, cur_bytes, hi = [], 0, off
            if cur:
                self._add_bucket(flat[off:hi], cur)
        self.pending = [0] * len(self.buckets)
        self.works = []
        for p in self.params:
            p.register_post_accumulate_grad_hook(self._ready)

    def _add_bucket(self, view, params):
        for p in params:
            self.bucket_of[id(p)] = len(self.buckets)
        self.buckets.append((view, params))

    def begin(self):
        for flat in self.flat.values():
            flat.zero_()
        self.pending = [len(ps) for _, ps in self.buckets]
        self.works = []

    def _reduce(self, b):
        import torch.distributed as dist
        view = self.buckets[b][0]
        if self.world > 1:
            view.mul_(1.0 / self.world)
        self.works.append(dist.all_reduce(view, group=self.group, async_op=True))

    def _ready(self, p):
        b = self.bucket_of[id(p)]
        self.pending[b] -= 1
        if self.pending[b] == 0:
            self._reduce(b)

    def finish(self):
        # A parameter that got no gradient this step (an unused branch or aux
        # head) never fired its hook: its bucket is reduced here, in bucket
        # order on every rank, so no replica is left with an unreduced bucket
        # (DDP's find_unused_parameters in effect).
        for b, left in enumerate(self.pending):
            if left > 0:
                self.pending[b] = 0
                self._reduce(b)
        for w in self.works:
            w.wait()
        self.works = []


def train(workload: str = "1.2", steps: int = 20, warmup: int = 5, bucket_mb: int = 64,
          backend: str | None = None, shrink: bool = False, batch: int | None = None,
          size: int | None = None, device: str | None = None, graph: bool | None = None) -> dict:
    import torch
    import torch.distributed as dist
    rank, world, device = setup(backend, device)
    torch.manual_seed(1234)
    w, model = build_model(workload, device, shrink=shrink)
    on_gpu = device.type == "cuda"
    collective_dev = on_gpu and dist.get_backend() == "nccl"
    with torch.no_grad():  # replicas start identical: rank 0's weights
        for t in list(model.parameters()) + list(model.buffers()):
            if collective_dev or t.device.type == "cpu":
                dist.broadcast(t.data, 0)
            else:
                c = t.data.cpu()
                dist.broadcast(c, 0)
                t.data.copy_(c)
    grads = GradBuckets(model.parameters(), bucket_mb, world)
    dtype = next(model.parameters()).dtype
    bsz = batch or w.batch
    shape = w.shape if size is None or w.kind != "image" else (w.shape[0], size, size)
    g = torch.Generator(device="cpu").manual_seed(100 + rank)   # each rank its own shard
    x = torch.randn((bsz, *shape), generator=g).to(device=device, dtype=dtype)
    if w.kind == "image":
        x = x.contiguous(memory_format=torch.channels_last)
    ncls = 10 if shrink else (21 if w.name == "deeplab" else (2 if w.name == "lstm" else 1000))
    tgt_shape = (bsz, *shape[1:]) if w.name == "deeplab" else (bsz,)
    tgt = torch.randint(0, ncls, tgt_shape, generator=g).to(device)
    opt = torch.optim.SGD(model.parameters(), lr=1e-3, momentum=0.9, fused=on_gpu or None)
    lossf = torch.nn.CrossEntropyLoss()

    def step():
        grads.begin()
        loss = lossf(model(x).float(), tgt)
        loss.backward()
        grads.finish()
        opt.step()
        return loss

    sync = torch.cuda.synchronize if on_gpu else (lambda: None)
    use_graph = collective_dev if graph is None else (graph and collective_dev)
    run = step
    captured = False
    if use_graph:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(max(warmup, 3)):  # communicator, MIOpen find, momentum buffers
                step()
        torch.cuda.current_stream().wait_stream(s)
        sync()
        try:
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                loss_static = step()
            captured = True

            def run():
                gr.replay()
                return loss_static
        except Exception as e:  # an op without capture support: eager steps
            if rank == 0:
                print(f"[ddp] step capture failed ({e}); eager", flush=True)
            sync()
    else:
        for _ in range(warmup):
            step()
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = run()
    sync()
    dist.barrier()
    dt = time.perf_counter() - t0
    red_dev = device if collective_dev else torch.device("cpu")
    t = torch.tensor([dt], dtype=torch.float64, device=red_dev)
    # every rank must end with the same weights (the all-reduce worked)
    chk = torch.stack([p.detach().float().sum() for p in model.parameters()]).sum().reshape(1).double().to(red_dev)
    chk_max, chk_min = chk.clone(), chk.clone()
    dist.all_reduce(chk_max, op=dist.ReduceOp.MAX)
    dist.all_reduce(chk_min, op=dist.ReduceOp.MIN)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall = float(t[0])
    return {"metric": "ddp training images/s", "workload": workload, "world": world,
            "value": round(bsz * world * steps / wall, 2), "unit": "images/s",
            "ms_per_step": round(1e3 * wall / steps, 3), "batch_per_rank": bsz, "bucket_mb": bucket_mb,
            "buckets": len(grads.buckets), "graph": captured, "backend": dist.get_backend(),
            "device": str(device), "dtype": str(dtype).replace("torch.", ""),
            "final_loss": float(loss.detach().float()),
            "weights_in_sync": bool(float(chk_max[0].item()) == float(chk_min[0].item()))}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="1.2")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--bucket-mb", type=int, default=64)
    ap.add_argument("--backend", default=None, help="nccl (RCCL) on GPU, gloo on CPU by default")
    ap.add_argument("--device", default=None, help="cuda: keep the model on the GPU even over gloo")
    ap.add_argument("--shrink", action="store_true", help="one-block-per-stage model (CPU rehearsal)")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--size", type=int, default=None)
    ap.add_argument("--no-graph", action="store_true", help="eager steps (default on GPU: one hipGraph per step)")
    args = ap.parse_args(argv)
    import torch.distributed as dist
    res = train(args.workload, args.steps, args.warmup, args.bucket_mb, args.backend, args.shrink,
                args.batch, args.size, args.device, graph=False if args.no_graph else None)
    if dist.get_rank() == 0:
        print(json.dumps(res), flush=True)
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
