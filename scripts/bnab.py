"""In-process A/B of the training BatchNorm reduction's shape
(native/kernels/bn_nhwc.hip, vgpu_bn_set_tuning): workgroups targeted over the
chip x rows in flight per thread, on every BatchNorm shape of a ResNet-V2-50
training step (ai-benchmark 1.2: b=20, 346²).  Forward (reduce + finalize +
apply) and backward (reduce + finalize + apply) per layer, interleaved.

    python scripts/bnab.py [--batch 20 --size 346] [--variants 1024x4,512x8,2048x4,1024x8]

One JSON line per shape plus totals.  Every variant's outputs are compared with
the first's (the reduction order changes, so up to bf16 rounding).

The timings are of eager autograd calls: on MI355X every shape measured
227-233 µs for every variant (round 4), i.e. the host's launch path, not the
kernels — use rocprofv3 kernel times to compare variants.  Since round 4 the
training path takes its BatchNorm statistics from the conv epilogues
(vgpu.ops.bnconv), so these reduction kernels run only where that does not
apply.
"""
from __future__ import annotations

import os as _os
import sys as _sys

_here = _os.path.dirname(_os.path.abspath(__file__))
_sys.path[:0] = [_here, _os.path.dirname(_here)]  # scripts/ and the repo root

import argparse
import json


def bn_shapes(batch: int, size: int) -> list[tuple[str, int, int, int]]:
    """(name, rows, channels, count) of the BatchNorms of a ResNet-V2-50 step."""
    s1 = (size + 1) // 2
    s1 = (s1 - 1) // 2 + 1                  # after the 3x3/s2 pool: 87 at 346
    hw = [s1, (s1 + 1) // 2, ((s1 + 1) // 2 + 1) // 2, (((s1 + 1) // 2 + 1) // 2 + 1) // 2]
    blocks, widths = [3, 4, 6, 3], [64, 128, 256, 512]
    out: dict[tuple[int, int], int] = {}
    cin = 64
    for st, (n, w) in enumerate(zip(blocks, widths)):
        for j in range(n):
            h_in = hw[st - 1] if (j == 0 and st > 0) else hw[st]
            out[(batch * h_in * h_in, cin)] = out.get((batch * h_in * h_in, cin), 0) + 1      # bn_in
            out[(batch * h_in * h_in, w)] = out.get((batch * h_in * h_in, w), 0) + 1          # bn1 (conv1 is 1x1/s1)
            out[(batch * hw[st] * hw[st], w)] = out.get((batch * hw[st] * hw[st], w), 0) + 1  # bn2
            cin = 4 * w
    out[(batch * hw[3] * hw[3], cin)] = out.get((batch * hw[3] * hw[3], cin), 0) + 1          # bn_out
    return [(f"m{m}c{c}", m, c, k) for (m, c), k in sorted(out.items(), key=lambda kv: -kv[0][0] * kv[0][1])]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=20)
    ap.add_argument("--size", type=int, default=346)
    ap.add_argument("--variants", default="1024x4,512x8,2048x4,1024x8")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args(argv)

    import torch
    from torch import nn
    from vgpu.native import load_kernels
    from vgpu.ops import bn as B
    from vgpu.utils.timing import interleaved_us
    lib = load_kernels()
    variants = [tuple(int(x) for x in v.split("x")) for v in args.variants.split(",")]
    tot = {v: 0.0 for v in variants}
    for name, m, c, count in bn_shapes(args.batch, args.size):
        # one image of m x 1 pixels: the same m rows of c channels as the real activation
        x = torch.randn(1, c, m, 1, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        bn = nn.BatchNorm2d(c).cuda()
        g = torch.randn_like(x)

        def mk(v):
            def f():
                lib.vgpu_bn_set_tuning(*v)
                xr = x.detach().requires_grad_(True)
                y = B.bn_act(xr, bn, "relu")
                y.backward(g)
                return xr.grad
            return f
        outs = {}
        for v in variants:
            outs[v] = mk(v)().float()
        us = interleaved_us([mk(v) for v in variants], rounds=args.rounds, iters=args.iters)
        lib.vgpu_bn_set_tuning(0, 0)
        row = {"shape": name, "rows": m, "C": c, "count": count, "MB": round(m * c * 2 / 1e6, 1)}
        ref = outs[variants[0]]
        for v, t in zip(variants, us):
            key = f"{v[0]}x{v[1]}"
            row[f"{key}_us"] = round(t, 1)
            row[f"{key}_maxdiff"] = round(float((outs[v] - ref).abs().max()), 4)
            tot[v] += t * count
        print(json.dumps(row), flush=True)
    print(json.dumps({"step_total_us": {f"{v[0]}x{v[1]}": round(t, 1) for v, t in tot.items()}}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
