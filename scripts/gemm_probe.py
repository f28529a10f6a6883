#!/usr/bin/env python3
"""One large 1x1 conv (= GEMM M x K x N) through the native conv path, for
rocprofv3 passes: python scripts/gemm_probe.py [big_mode] [M] [K] [N] [iters]
(big_mode: 1 = 256x256 tile, 0 = 128x128 kernels)."""
import sys

import torch

from vgpu.native import load_kernels
from vgpu.ops import conv as C

mode, m, k, n, iters = (int(v) for v in (sys.argv[1:] + ["1", "65536", "1024", "1024", "20"][len(sys.argv) - 1:]))
side = int(m ** 0.5)
x = torch.randn(m // side, k, side, 1, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
x = torch.randn(1, k, m // side, side, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
w = (torch.randn(n, k, 1, 1, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
load_kernels().vgpu_conv_set_big(mode)
for _ in range(iters):
    C.conv2d(x, w)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(iters):
    C.conv2d(x, w)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / iters
print(f"GEMM mode={mode} M={m} K={k} N={n}: {us:.1f} us, {2.0 * m * k * n / us / 1e6:.0f} TFLOP/s", flush=True)
