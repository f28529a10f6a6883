#!/usr/bin/env python3
"""Which Python lines launch a training step's PyTorch kernels: one eager step
of an ai-benchmark workload under torch.profiler (with_stack), aten ops that
reached the GPU grouped by their innermost frames under vgpu/.

    python scripts/step_attrib.py --workload 4.2 > gpurun_out/attrib_4_2.txt
"""
from __future__ import annotations

import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="4.2")
    a = ap.parse_args()
    from vgpu.bench import pod
    ns = argparse.Namespace(workload=a.workload, pod_index=0, find=False, graph=False, no_fused=False,
                            conv="native", train_graph=False)
    _, step = pod.build(ns)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    # kernels per launching aten op, keyed by (op, first vgpu/ frames)
    by = collections.Counter()
    kern = collections.Counter()
    evs = prof.events()
    for e in evs:
        if e.device_type == torch.autograd.DeviceType.CUDA:
            kern[e.name[:90]] += 1
    for e in evs:
        if e.device_type != torch.autograd.DeviceType.CPU or not e.name.startswith("aten::"):
            continue
        nk = len([k for k in e.kernels]) if hasattr(e, "kernels") else 0
        if not nk:
            continue
        if any(p.name.startswith("aten::") for p in [e.cpu_parent] if p is not None):
            continue  # count at the outermost aten op
        fr = [s for s in (e.stack or []) if "vgpu/" in s or "scripts/" in s or "torch/autograd" in s][:3]
        by[(e.name, " <- ".join(fr))] += nk
    print(f"{sum(kern.values())} kernels in one eager step\n")
    for (op, fr), n in by.most_common(60):
        print(f"{n:5d}  {op:32s} {fr}")
    print("\n-- kernels --")
    for k, n in kern.most_common(40):
        print(f"{n:5d}  {k}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
