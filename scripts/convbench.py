"""Micro-benchmark of ResNet-V2-50 layer shapes (b=50, 346²) on MI355X:
MIOpen conv (channels_last) vs GEMM formulations, and elementwise passes.
Prints one JSON line per case.  python scripts/convbench.py
"""
from __future__ import annotations

import os as _os
import sys as _sys

_here = _os.path.dirname(_os.path.abspath(__file__))
_sys.path[:0] = [_here, _os.path.dirname(_here)]  # scripts/ and the repo root

import json
import sys

import torch
import torch.nn.functional as F


def timeit(fn, reps=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def main() -> int:
    find = "--find" in sys.argv
    torch.backends.cudnn.benchmark = find
    dev = "cuda"
    B = 50
    # (H, Cin, Cout, k, stride)
    cases = [(87, 64, 64, 1, 1), (87, 64, 256, 1, 1), (87, 256, 64, 1, 1), (87, 64, 64, 3, 1),
             (44, 128, 128, 3, 1), (44, 128, 512, 1, 1), (44, 512, 128, 1, 1),
             (22, 256, 256, 3, 1), (22, 256, 1024, 1, 1), (22, 1024, 256, 1, 1),
             (11, 512, 512, 3, 1), (11, 512, 2048, 1, 1), (11, 2048, 512, 1, 1)]
    for H, ci, co, k, s in cases:
        x = torch.randn(B, ci, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = torch.randn(co, ci, k, k, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        bias = torch.randn(co, device=dev, dtype=torch.bfloat16)
        t_conv = timeit(lambda: F.conv2d(x, w, padding=k // 2, stride=s))
        t_convb = timeit(lambda: F.relu(F.conv2d(x, w, bias, padding=k // 2, stride=s)))
        res = {"H": H, "cin": ci, "cout": co, "k": k, "conv_us": round(t_conv, 1),
               "conv_bias_relu_us": round(t_convb, 1)}
        flops = 2 * B * H * H * ci * co * k * k
        res["conv_tflops"] = round(flops / t_conv / 1e6, 1)
        if k == 1:
            a = x.permute(0, 2, 3, 1).reshape(-1, ci)
            wt = w.reshape(co, ci)
            t_mm = timeit(lambda: a @ wt.t())
            t_addmm = timeit(lambda: torch.addmm(bias, a, wt.t()))
            t_act = timeit(lambda: torch._addmm_activation(bias, a, wt.t()))
            res.update({"mm_us": round(t_mm, 1), "addmm_us": round(t_addmm, 1),
                        "addmm_relu_us": round(t_act, 1), "mm_tflops": round(flops / t_mm / 1e6, 1)})
        y = torch.randn(B, co, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        res["relu_us"] = round(timeit(lambda: F.relu(y)), 1)
        res["bytes_out_MB"] = round(y.numel() * 2 / 1e6, 1)
        print("CASE " + json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
