"""In-process A/B of two builds of the native convolution (box-to-box variance
is ±10 % per layer, so kernel changes are judged in one process).

    python scripts/convab.py --other vgpu/_lib/libvgpu_conv_ab.so [--batch 50 --size 346]

`--other` is a shared library exporting the same `vgpu_conv2d_nhwc` /
`vgpu_conv23_nhwc` ABI (e.g. the previous commit's conv_gemm.hip built alone);
the current build is vgpu/_lib/libvgpu_kernels.so.  Every flagship layer (and
the fused bottleneck tails) runs alternately on both, 3 rounds, and one JSON
line per layer reports both times.
"""
from __future__ import annotations

import os as _os
import sys as _sys

_here = _os.path.dirname(_os.path.abspath(__file__))
_sys.path[:0] = [_here, _os.path.dirname(_here)]  # scripts/ and the repo root

import argparse
import ctypes
import json

from convnative import layer_shapes  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--other", required=True)
    ap.add_argument("--batch", type=int, default=50)
    ap.add_argument("--size", type=int, default=346)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args(argv)

    import torch
    from vgpu.native import load_kernels
    from vgpu.ops import conv as C
    cur = load_kernels()
    old = ctypes.CDLL(args.other)
    vp, ci = ctypes.c_void_p, ctypes.c_int
    old.vgpu_conv2d_nhwc.argtypes = [vp] * 7 + [ci] * 9 + [vp]
    cl = torch.channels_last
    dev = "cuda"
    P = C._ptr

    from vgpu.utils.timing import cuda_time_us

    def timeit(fn):
        return cuda_time_us(fn, args.iters)

    tot = [0.0, 0.0]
    for name, n, c, h, w, cout, ks, stride, pad, ba, pro, res in layer_shapes(args.batch, args.size):
        x = torch.randn(n, c, h, w, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        wt = (torch.randn(cout, c, ks, ks, device=dev) * (2 / (c * ks * ks)) ** 0.5).to(
            torch.bfloat16).contiguous(memory_format=cl)
        oh, ow = C.out_hw(h, w, ks, stride, pad)
        bias = torch.zeros(cout, device=dev) if ba else None
        pp = (torch.ones(c, device=dev), torch.zeros(c, device=dev)) if pro else None
        r = torch.randn(n, cout, oh, ow, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl) if res else None
        ys = [torch.empty(n, cout, oh, ow, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
              for _ in range(2)]

        def run(lib, y):
            rc = lib.vgpu_conv2d_nhwc(P(x), P(wt), P(y), P(r), P(bias), P(pp[0] if pp else None),
                                      P(pp[1] if pp else None), n, h, w, c, cout, ks, stride, pad,
                                      1 if ba else 0, C._stream())
            assert rc == 0, rc
        t = [0.0, 0.0]
        for _ in range(3):
            t[0] += timeit(lambda: run(cur, ys[0])) / 3
            t[1] += timeit(lambda: run(old, ys[1])) / 3
        same = bool(torch.equal(ys[0], ys[1]))
        tot[0] += t[0]
        tot[1] += t[1]
        print(json.dumps({"layer": name, "new_us": round(t[0], 1), "old_us": round(t[1], 1),
                          "bit_exact": same}), flush=True)
    h1 = ((args.size + 6 - 7) // 2 + 1 + 2 - 3) // 2 + 1
    if hasattr(old, "vgpu_conv23_nhwc"):
        for name, c, h, stride in (("s1.tail", 64, h1, 1), ("s2b1.tail", 128, h1, 2),
                                   ("s2.tail", 128, (h1 - 1) // 2 + 1, 1)):
            n = args.batch
            x = torch.randn(n, c, h, h, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
            w2 = (torch.randn(c, c, 3, 3, device=dev) * (2 / (9 * c)) ** 0.5).to(torch.bfloat16).contiguous(
                memory_format=cl)
            b2 = torch.zeros(c, device=dev)
            w3 = (torch.randn(4 * c, c, 1, 1, device=dev) * (2 / c) ** 0.5).to(torch.bfloat16).contiguous(
                memory_format=cl)
            oh = (h - 1) // stride + 1
            r = torch.randn(n, 4 * c, oh, oh, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
            ys = [torch.empty_like(r) for _ in range(2)]

            def run23(lib, y):
                rc = lib.vgpu_conv23_nhwc(P(x), P(w2), P(b2), P(w3), P(r), P(y), n, h, h, c, stride, C._stream())
                assert rc == 0, rc
            t = [0.0, 0.0]
            for _ in range(3):
                t[0] += timeit(lambda: run23(cur, ys[0])) / 3
                t[1] += timeit(lambda: run23(old, ys[1])) / 3
            tot[0] += t[0]
            tot[1] += t[1]
            print(json.dumps({"layer": name, "new_us": round(t[0], 1), "old_us": round(t[1], 1),
                              "bit_exact": bool(torch.equal(ys[0], ys[1]))}), flush=True)
            if not hasattr(old, "vgpu_conv231_nhwc"):
                continue
            # + the next identity block's BN+ReLU+conv1 (conv231, stride-1 shapes)
            w1n = (torch.randn(c, 4 * c, 1, 1, device=dev) * (2 / (4 * c)) ** 0.5).to(
                torch.bfloat16).contiguous(memory_format=cl)
            b1n = torch.zeros(c, device=dev)
            ps, pt = torch.rand(4 * c, device=dev) + 0.5, torch.randn(4 * c, device=dev) * 0.1
            hs = [torch.empty(n, c, oh, oh, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
                  for _ in range(2)]

            def run231(lib, y, h1):
                rc = lib.vgpu_conv231_nhwc(P(x), P(w2), P(b2), P(w3), P(r), P(y), P(w1n), P(b1n), P(ps), P(pt),
                                           P(h1), n, h, h, c, stride, C._stream())
                assert rc == 0, rc
            t = [0.0, 0.0]
            for _ in range(3):
                t[0] += timeit(lambda: run231(cur, ys[0], hs[0])) / 3
                t[1] += timeit(lambda: run231(old, ys[1], hs[1])) / 3
            tot[0] += t[0]
            tot[1] += t[1]
            print(json.dumps({"layer": name.replace("tail", "tail+next"), "new_us": round(t[0], 1),
                              "old_us": round(t[1], 1),
                              "bit_exact": bool(torch.equal(ys[0], ys[1]) and torch.equal(hs[0], hs[1]))}),
                  flush=True)
    print(json.dumps({"total_new_us": round(tot[0], 1), "total_old_us": round(tot[1], 1)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
