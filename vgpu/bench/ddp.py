"""Data-parallel training inside ONE multi-GPU vGPU pod.

The pod is admitted through the control plane with `amd.com/gpu: N`
(vgpu.bench.control.admit_multi_gpu_pod): Allocate hands it N devices, each
with its own cap / compute share, and one shared region for the container.
Inside it, torchrun starts one rank per visible device; every rank runs the
ai-benchmark ResNet-V2-50 training step (test 1.2: batch 20, 346², bf16,
channels_last, the native MFMA convolutions) under DistributedDataParallel
over RCCL, with the enforcement library preloaded in every rank.

    python -m torch.distributed.run --nproc-per-node N -m vgpu.bench.ddp --steps K --warmup W

Rank 0 prints one line `DDP {json}`: aggregate images/s over all ranks, the
max step time over ranks, and the gradient bucket size.  The launcher
(bench.py --pod-gpus) parses RCCL's chosen transport per peer from
NCCL_DEBUG=INFO.  --cpu-smoke rehearses the same orchestration on CPU (gloo,
a small input) for tests; it is not a measurement.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="1.2")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--bucket-mb", type=int, default=100,
                    help="DDP gradient bucket (MiB): few large all-reduces suit ring collectives over xGMI")
    ap.add_argument("--cpu-smoke", action="store_true")
    args = ap.parse_args(argv)

    import torch
    import torch.distributed as dist
    from torch.nn.parallel import DistributedDataParallel as DDP

    from vgpu.models import WORKLOADS

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    w = WORKLOADS[args.workload]
    if not w.train:
        raise SystemExit(f"workload {args.workload} is not a training test")
    if args.cpu_smoke:
        dev = torch.device("cpu")
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dtype = torch.float32
        batch, shape = 2, (3, 64, 64)
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        dtype = torch.bfloat16
        batch, shape = w.batch, tuple(w.shape)
    torch.manual_seed(1234)  # identical initial weights on every rank
    model = w.builder().to(dev).to(dtype)
    if not args.cpu_smoke:
        model = model.to(memory_format=torch.channels_last)
    model.train()
    ddp = DDP(model, device_ids=None if args.cpu_smoke else [local], bucket_cap_mb=args.bucket_mb,
              gradient_as_bucket_view=True)
    opt = torch.optim.SGD(ddp.parameters(), lr=1e-3, momentum=0.9,
                          fused=None if args.cpu_smoke else True)
    g = torch.Generator(device="cpu").manual_seed(100 + rank)  # each rank its own shard of synthetic data
    x = torch.randn((batch, *shape), generator=g).to(dev, dtype)
    if not args.cpu_smoke:
        x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (batch,), generator=g).to(dev)
    lossf = torch.nn.CrossEntropyLoss()
    sync = (lambda: None) if args.cpu_smoke else torch.cuda.synchronize

    def step():
        opt.zero_grad(set_to_none=True)
        loss = lossf(ddp(x).float(), y)
        loss.backward()
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    sync()
    dist.barrier()
    sync()
    t0 = time.monotonic()
    for _ in range(args.steps):
        loss = step()
    sync()
    dist.barrier()
    sync()
    dt = time.monotonic() - t0
    t = torch.tensor([dt, float(loss.detach().float())], dtype=torch.float64, device=dev)
    mx = t.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    # the replicas must agree after identical all-reduced updates
    p0 = next(ddp.parameters()).detach().float().sum().reshape(1).to(torch.float64)
    pmin, pmax = p0.clone(), p0.clone()
    dist.all_reduce(pmin, op=dist.ReduceOp.MIN)
    dist.all_reduce(pmax, op=dist.ReduceOp.MAX)
    if rank == 0:
        wall = float(mx[0])
        out = {"world": world, "steps": args.steps, "warmup": args.warmup, "batch_per_rank": batch,
               "ms_per_step": round(1e3 * wall / max(args.steps, 1), 3),
               "images_per_s": round(world * batch * args.steps / max(wall, 1e-9), 2),
               "bucket_mb": args.bucket_mb, "backend": dist.get_backend(),
               "replicas_agree": bool(abs(float(pmax) - float(pmin)) <= 1e-3 * max(1.0, abs(float(pmax)))),
               "loss": round(float(t[1]), 4), "dtype": str(dtype).replace("torch.", "")}
        sys.stdout.write("DDP " + json.dumps(out) + "\n")
        sys.stdout.flush()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
