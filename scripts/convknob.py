"""In-process A/B of the native convolution's dispatch knobs on one layer set
(box-to-box variance is ±10 % per kernel, so variants are compared in one
process, interleaved).

    python scripts/convknob.py [--knob halo] [--batch 50 --size 346] [--extra]

--knob halo: 3x3 / stride-1 layers with the halo-tile kernel off (LDS-DMA
per-tap gathers), on (heuristic tile) and forced to 256- / 128-row tiles
(native/kernels/conv_gemm.hip conv_halo_kernel).  --extra adds the
ResNet-V2-152 (b=10, 256²) and ResNet-V2-50 training (b=20) 3x3 shapes.
One JSON line per layer: µs and TFLOP/s per variant.
"""
from __future__ import annotations

import os as _os
import sys as _sys

_here = _os.path.dirname(_os.path.abspath(__file__))
_sys.path[:0] = [_here, _os.path.dirname(_here)]  # scripts/ and the repo root

import argparse
import json

from convnative import layer_shapes  # noqa: E402

KNOBS = {
    # name: (setter, [(tag, value)])
    "halo": ("vgpu_conv_set_halo", [("off", 0), ("auto", -1), ("bm256", 2), ("bm128", 3)]),
}


def halo_layers(batch: int, size: int, extra: bool):
    out = [s for s in layer_shapes(batch, size) if s[6] == 3 and s[7] == 1]
    if extra:
        out += [(f"r152.{s[0]}", *s[1:]) for s in layer_shapes(10, 256) if s[6] == 3 and s[7] == 1]
        out += [(f"train.{s[0]}", *s[1:]) for s in layer_shapes(20, size) if s[6] == 3 and s[7] == 1]
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--knob", default="halo", choices=sorted(KNOBS))
    ap.add_argument("--batch", type=int, default=50)
    ap.add_argument("--size", type=int, default=346)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--extra", action="store_true")
    args = ap.parse_args(argv)

    import torch
    from vgpu.native import load_kernels
    from vgpu.ops import conv as C
    from vgpu.utils.timing import interleaved_us
    lib = load_kernels()
    setter_name, variants = KNOBS[args.knob]
    setter = getattr(lib, setter_name)
    cl = torch.channels_last
    tot = {tag: 0.0 for tag, _ in variants}
    for name, n, c, h, w, cout, ks, stride, pad, ba, pro, res in halo_layers(args.batch, args.size, args.extra):
        x = torch.randn(n, c, h, w, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)
        wt = (torch.randn(cout, c, ks, ks, device="cuda") * (2 / (c * ks * ks)) ** 0.5).to(
            torch.bfloat16).contiguous(memory_format=cl)
        bias = torch.zeros(cout, device="cuda") if ba else None
        oh, ow = C.out_hw(h, w, ks, stride, pad)
        y = torch.empty(n, cout, oh, ow, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)

        def mk(v):
            def f():
                setter(v)
                C.conv2d(x, wt, bias, stride=stride, padding=pad, act="relu" if ba else "none", out=y)
            return f
        ref = None
        outs = {}
        for tag, v in variants:  # correctness of every variant against the first
            mk(v)()
            outs[tag] = y.float().clone()
            ref = outs[variants[0][0]]
        us = interleaved_us([mk(v) for _, v in variants], rounds=args.rounds, iters=args.iters)
        setter(-1)
        flop = 2.0 * n * oh * ow * cout * c * ks * ks
        row = {"layer": name, "M": n * oh * ow, "K": c * ks * ks, "N": cout}
        for (tag, _), t in zip(variants, us):
            row[f"{tag}_us"] = round(t, 1)
            row[f"{tag}_tflops"] = round(flop / t / 1e6, 1)
            row[f"{tag}_maxdiff"] = round(float((outs[tag] - ref).abs().max()), 4)
            tot[tag] += t
        print(json.dumps(row), flush=True)
    print(json.dumps({"total_us": {k: round(v, 1) for k, v in tot.items()}}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
