"""Per-layer timing of the MFMA implicit-GEMM convolution against MIOpen on the
ResNet-V2-50 layer shapes of ai-benchmark test 1.1 (b=50, 346²).

    python scripts/convnative.py [--batch 50 --size 346 --iters 20]

Prints one JSON line per layer: native µs (with its fused prologue/epilogue),
MIOpen µs (bare convolution after find), TFLOP/s, and the native kernel's
effective HBM bandwidth (compulsory bytes / time).
"""
from __future__ import annotations

import os as _os
import sys as _sys

_here = _os.path.dirname(_os.path.abspath(__file__))
_sys.path[:0] = [_here, _os.path.dirname(_here)]  # scripts/ and the repo root

import argparse
import json


def layer_shapes(batch: int, size: int):
    """(name, n, c, h, w, cout, ks, stride, pad, bias/act, prologue, residual) of every
    distinct convolution after the stem."""
    h = ((size + 6 - 7) // 2 + 1 + 2 - 3) // 2 + 1
    cin = 64
    out = []
    for i, (n_blocks, width) in enumerate(zip((3, 4, 6, 3), (64, 128, 256, 512))):
        for j in range(min(n_blocks, 2)):
            stride = 2 if (j == 0 and i > 0) else 1
            cout = width * 4
            tag = f"s{i + 1}b{j + 1}"
            oh = (h + 2 - 3) // stride + 1
            if j == 0:
                out.append((f"{tag}.sc", batch, cin, h, h, cout, 1, stride, 0, False, True, False))
            out.append((f"{tag}.conv1", batch, cin, h, h, width, 1, 1, 0, True, True, False))
            out.append((f"{tag}.conv2", batch, width, h, h, width, 3, stride, 1, True, False, False))
            out.append((f"{tag}.conv3", batch, width, oh, oh, cout, 1, 1, 0, False, False, True))
            h, cin = oh, cout
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=50)
    ap.add_argument("--size", type=int, default=346)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--no-miopen", action="store_true")
    ap.add_argument("--only", default="", help="comma-separated layer names (profiling)")
    ap.add_argument("--no-stem", action="store_true")
    ap.add_argument("--ab-tail", action="store_true",
                    help="bottleneck tail conv2+conv3: fused kernel vs the two kernels (stages 1-2)")
    ap.add_argument("--ab-tile", action="store_true",
                    help="per layer, interleaved: 64-row vs 128-row tiles")
    args = ap.parse_args(argv)

    import torch
    import torch.nn.functional as F
    from vgpu.ops import conv as C
    torch.backends.cudnn.benchmark = True
    cl = torch.channels_last
    dev = "cuda"

    from vgpu.utils.timing import cuda_time_us

    def timeit(fn):
        return cuda_time_us(fn, args.iters)

    tot_n = tot_m = 0.0
    if args.ab_tail:
        return _ab_tail(args, timeit, C, cl, dev)
    only = set(filter(None, args.only.split(",")))
    if args.no_stem or only:
        layers = [l for l in layer_shapes(args.batch, args.size) if not only or l[0] in only]
        return _run_layers(args, layers, timeit, C, F, cl, dev)
    # stem: space-to-depth + 4x4 narrow-C MFMA conv vs MIOpen's 7x7/s2 on C=3
    xs = torch.randn(args.batch, 3, args.size, args.size, device=dev, dtype=torch.bfloat16).contiguous(
        memory_format=cl)
    ws = (torch.randn(64, 3, 7, 7, device=dev) * (2 / 147) ** 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
    ws2d = C.stem_weight_s2d(ws)
    t_nat = timeit(lambda: C.stem_conv(xs, ws2d))
    t_mio = None if args.no_miopen else timeit(lambda: F.conv2d(xs, ws, stride=2, padding=3))
    oh = (args.size + 6 - 7) // 2 + 1
    flop = 2.0 * args.batch * oh * oh * 64 * 147
    tot_n += t_nat
    tot_m += t_mio or 0.0
    print(json.dumps({"layer": "stem", "M": args.batch * oh * oh, "K": 147, "N": 64,
                      "native_us": round(t_nat, 1), "miopen_us": None if t_mio is None else round(t_mio, 1),
                      "native_tflops": round(flop / t_nat / 1e6, 1),
                      "native_tbps": round((xs.numel() * 2 + args.batch * oh * oh * 64 * 2) / t_nat / 1e6, 2)}),
          flush=True)
    y0 = C.stem_conv(xs, ws2d)
    t_pool = timeit(lambda: C.maxpool3s2(y0))
    print(json.dumps({"layer": "stem.maxpool", "native_us": round(t_pool, 1),
                      "native_tbps": round((y0.numel() * 2 * 1.25) / t_pool / 1e6, 2)}), flush=True)
    tot_n += t_pool
    return _run_layers(args, layer_shapes(args.batch, args.size), timeit, C, F, cl, dev, tot_n, tot_m)


def _ab_tail(args, timeit, C, cl, dev) -> int:
    import torch
    h1 = ((args.size + 6 - 7) // 2 + 1 + 2 - 3) // 2 + 1
    for name, c, h, stride in (("s1.tail", 64, h1, 1), ("s2b1.tail", 128, h1, 2),
                               ("s2.tail", 128, (h1 - 1) // 2 + 1, 1)):
        n = args.batch
        x = torch.randn(n, c, h, h, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        w2 = (torch.randn(c, c, 3, 3, device=dev) * (2 / (9 * c)) ** 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
        b2 = torch.zeros(c, device=dev)
        w3 = (torch.randn(4 * c, c, 1, 1, device=dev) * (2 / c) ** 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
        oh = (h - 1) // stride + 1
        r = torch.randn(n, 4 * c, oh, oh, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        y = torch.empty_like(r)
        two = lambda: C.conv2d(C.conv2d(x, w2, b2, stride=stride, padding=1, act="relu"), w3,  # noqa: E731
                               residual=r, out=y)
        one = lambda: C.conv23(x, w2, b2, w3, r, stride=stride, out=y)  # noqa: E731
        tf = tu = 0.0
        for _ in range(3):
            tu += timeit(two) / 3
            tf += timeit(one) / 3
        print(json.dumps({"layer": name, "unfused_us": round(tu, 1), "fused_us": round(tf, 1)}), flush=True)
    return 0


def _run_layers(args, layers, timeit, C, F, cl, dev, tot_n=0.0, tot_m=0.0) -> int:
    import torch
    for name, n, c, h, w, cout, ks, stride, pad, ba, pro, res in layers:
        x = torch.randn(n, c, h, w, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        wt = (torch.randn(cout, c, ks, ks, device=dev) * (2 / (c * ks * ks)) ** 0.5).to(
            torch.bfloat16).contiguous(memory_format=cl)
        oh, ow = C.out_hw(h, w, ks, stride, pad)
        bias = torch.zeros(cout, device=dev) if ba else None
        pp = (torch.ones(c, device=dev), torch.zeros(c, device=dev)) if pro else None
        r = torch.randn(n, cout, oh, ow, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl) if res else None
        y = torch.empty(n, cout, oh, ow, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        t_nat = timeit(lambda: C.conv2d(x, wt, bias, stride=stride, padding=pad,
                                        act="relu" if ba else "none", pro=pp, residual=r, out=y))
        if args.ab_tile:
            from vgpu.native import load_kernels
            lib = load_kernels()
            run = lambda: C.conv2d(x, wt, bias, stride=stride, padding=pad,  # noqa: E731
                                   act="relu" if ba else "none", pro=pp, residual=r, out=y)
            t64 = t128 = 0.0
            for _ in range(3):
                lib.vgpu_conv_set_tile_m(64)
                t64 += timeit(run) / 3
                lib.vgpu_conv_set_tile_m(128)
                t128 += timeit(run) / 3
            lib.vgpu_conv_set_tile_m(0)
            print(json.dumps({"layer": name, "bm64_us": round(t64, 1), "bm128_us": round(t128, 1)}), flush=True)
        t_mio = None if args.no_miopen else timeit(lambda: F.conv2d(x, wt, stride=stride, padding=pad))
        flop = 2.0 * n * oh * ow * cout * c * ks * ks
        in_bytes = x.numel() * 2 if (ks == 1 and stride == 1) or ks == 3 else n * oh * ow * c * 2
        nbytes = in_bytes + wt.numel() * 2 + y.numel() * 2 * (2 if res else 1)
        tot_n += t_nat
        tot_m += t_mio or 0.0
        print(json.dumps({"layer": name, "M": n * oh * ow, "K": c * ks * ks, "N": cout,
                          "native_us": round(t_nat, 1),
                          "miopen_us": None if t_mio is None else round(t_mio, 1),
                          "native_tflops": round(flop / t_nat / 1e6, 1),
                          "native_tbps": round(nbytes / t_nat / 1e6, 2)}), flush=True)
    print(json.dumps({"total_native_us": round(tot_n, 1), "total_miopen_us": round(tot_m, 1)}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
