"""Data-parallel training of the ai-benchmark training workloads, one process
per (v)GPU, gradients all-reduced over RCCL (torch.distributed backend "nccl"
is RCCL on ROCm) — the multi-GPU data-plane of SURVEY.md §2.9 ("benchmark
harness only: PyTorch DDP over RCCL/xGMI for the 1/2/4/8-GPU scaling curve;
the shim must not break RCCL").

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        -m vgpu.parallel.ddp --workload 1.2 --steps 20 --warmup 5

Design for MI355X over xGMI (7 point-to-point links per GPU, ≈153 GB/s each):
ring all-reduce is per-link bound, so gradients go in few, large buckets
(`--bucket-mb`, default 64 MB: a ResNet-V2-50 bf16 step is ~50 MB of
gradients, i.e. one or two collectives instead of DDP's default 25 MB chunks),
launched as soon as each bucket's gradients are ready so the collective
overlaps the rest of the backward pass.  Gradients are reduced in bf16 (the
model dtype) with gradient-as-bucket-view (no copy into the bucket).  Each
rank runs the same native kernels as a single pod (vgpu.ops.bn / conv) and,
under the enforcement library, its pod's CU mask and HBM cap; RCCL's own
kernels are exempt from the temporal limiter (native/shim/limiter.cpp).

On CPU (tests) the same code runs over gloo.  Prints one JSON line on rank 0:
aggregate images/s over all ranks (max step time over ranks).
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
        dist.init_process_group(backend or ("nccl" if use_gpu else "gloo"), rank=rank, world_size=world)
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


def wrap(model, device, bucket_mb: int = 64):
    import torch
    from torch.nn.parallel import DistributedDataParallel as DDP
    return DDP(model, device_ids=[device.index] if device.type == "cuda" else None,
               bucket_cap_mb=bucket_mb, gradient_as_bucket_view=True, static_graph=True,
               broadcast_buffers=False, find_unused_parameters=False)


def train(workload: str = "1.2", steps: int = 20, warmup: int = 5, bucket_mb: int = 64,
          backend: str | None = None, shrink: bool = False, batch: int | None = None,
          size: int | None = None, device: str | None = None) -> dict:
    import torch
    import torch.distributed as dist
    rank, world, device = setup(backend, device)
    torch.manual_seed(1234)  # identical initial weights on every rank (DDP also broadcasts)
    w, model = build_model(workload, device, shrink=shrink)
    ddp = wrap(model, device, bucket_mb)
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
    fused = device.type == "cuda"
    opt = torch.optim.SGD(ddp.parameters(), lr=1e-3, momentum=0.9, fused=fused or None)
    lossf = torch.nn.CrossEntropyLoss()

    def step():
        opt.zero_grad(set_to_none=False)
        loss = lossf(ddp(x).float(), tgt)
        loss.backward()
        opt.step()
        return loss

    sync = torch.cuda.synchronize if device.type == "cuda" else (lambda: None)
    for _ in range(warmup):
        step()
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    sync()
    dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=device if backend != "gloo" and device.type == "cuda" else "cpu")
    # every rank must end with the same weights (the all-reduce worked)
    chk = torch.stack([p.detach().float().sum() for p in model.parameters()]).sum().reshape(1).double()
    chk = chk if dist.get_backend() == "nccl" else chk.cpu()  # RCCL reduces device tensors only
    chk_max, chk_min = chk.clone(), chk.clone()
    dist.all_reduce(chk_max, op=dist.ReduceOp.MAX)
    dist.all_reduce(chk_min, op=dist.ReduceOp.MIN)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall = float(t[0])
    res = {"metric": "ddp training images/s", "workload": workload, "world": world,
           "value": round(bsz * world * steps / wall, 2), "unit": "images/s",
           "ms_per_step": round(1e3 * wall / steps, 3), "bucket_mb": bucket_mb,
           "backend": dist.get_backend(), "device": str(device), "final_loss": float(loss.detach().float()),
           "weights_in_sync": bool(float(chk_max[0].item()) == float(chk_min[0].item()))}
    return res


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
    args = ap.parse_args(argv)
    import torch.distributed as dist
    res = train(args.workload, args.steps, args.warmup, args.bucket_mb, args.backend, args.shrink,
                args.batch, args.size, args.device)
    if dist.get_rank() == 0:
        print(json.dumps(res), flush=True)
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
