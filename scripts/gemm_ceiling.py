#!/usr/bin/env python3
"""Library ceiling for the GEMM shapes inside ResNet-V2-50's convolutions:
hipBLASLt (torch.mm, bf16) TFLOP/s on M x K x N = the implicit-GEMM view of a
layer, next to the native conv kernel's time for the same layer.

    python scripts/gemm_ceiling.py [--iters 50]
"""
from __future__ import annotations

import argparse
import json


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    import torch
    from vgpu.ops import conv as C
    cl = torch.channels_last

    def timeit(fn):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / args.iters

    # (name, n, c, h, cout, ks, stride, pad) at b=50, 346² input
    shapes = [("s3.conv1", 50, 1024, 22, 256, 1, 1, 0), ("s3.conv2", 50, 256, 22, 256, 3, 1, 1),
              ("s4.conv1", 50, 2048, 11, 512, 1, 1, 0), ("s4.conv2", 50, 512, 11, 512, 3, 1, 1),
              ("s2.conv3", 50, 128, 44, 512, 1, 1, 0), ("big", 64, 1024, 32, 1024, 1, 1, 0),
              ("big4k", 64, 4096, 32, 4096, 1, 1, 0)]
    for name, n, c, h, cout, ks, stride, pad in shapes:
        oh = (h + 2 * pad - ks) // stride + 1
        m, k = n * oh * oh, c * ks * ks
        a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
        b = torch.randn(k, cout, device="cuda", dtype=torch.bfloat16)
        t_mm = timeit(lambda: torch.mm(a, b))
        x = torch.randn(n, c, h, h, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)
        w = (torch.randn(cout, c, ks, ks, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=cl)
        t_nat = timeit(lambda: C.conv2d(x, w, stride=stride, padding=pad))
        flop = 2.0 * m * k * cout
        extra = {}
        if ks == 1 and stride == 1 and cout % 256 == 0:  # 128x128 kernels vs the 256x256 tile
            from vgpu.native import load_kernels
            lib = load_kernels()
            lib.vgpu_conv_set_big(0)
            t_128 = timeit(lambda: C.conv2d(x, w, stride=stride, padding=pad))
            lib.vgpu_conv_set_big(1)
            t_256 = timeit(lambda: C.conv2d(x, w, stride=stride, padding=pad))
            lib.vgpu_conv_set_big(-1)
            extra = {"tile128_tflops": round(flop / t_128 / 1e6), "tile256_tflops": round(flop / t_256 / 1e6)}
        print(json.dumps({"layer": name, "M": m, "K": k, "N": cout,
                          "hipblaslt_us": round(t_mm, 1), "hipblaslt_tflops": round(flop / t_mm / 1e6),
                          "native_us": round(t_nat, 1), "native_tflops": round(flop / t_nat / 1e6), **extra}),
              flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
