#!/usr/bin/env python3
"""The flagship's conv shapes (ResNet-V2-50 inference, b=50, 346²) on the
native kernels against hipBLASLt on the same GEMM.

Each row: one layer's implicit-GEMM view M x K x N; the native conv2d as the
inference forward calls it (BN+ReLU prologue / residual as in the model), and
torch.mm (hipBLASLt) of an M x K by K x N bf16 GEMM -- for a 3x3 conv K = 9C,
i.e. hipBLASLt is handed an already-materialised im2col it does not have to
build, a ceiling in its favour.  Both are timed as 20 launches replayed from
one hipGraph, in-process.  conv23 (conv2 + conv3 + residual fused) is compared
with the two hipBLASLt GEMMs it replaces.

    python scripts/family_vs_hipblaslt.py > profiles/r6/kernels/family_vs_hipblaslt.json
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CL = torch.channels_last


def graph_us(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (3 * reps)


def main() -> int:
    from vgpu.ops import conv as C
    dev = "cuda"
    b = 50
    # (family, name, C, H, Cout, ks, stride, prologue, residual)
    layers = [
        ("conv_pro", "s1 conv1 256->64 @87", 256, 87, 64, 1, 1, True, False),
        ("conv_pro", "s2 conv1 512->128 @44", 512, 44, 128, 1, 1, True, False),
        ("conv_pro", "s3 conv1 1024->256 @22", 1024, 22, 256, 1, 1, True, False),
        ("conv_pro", "s4 conv1 2048->512 @11", 2048, 11, 512, 1, 1, True, False),
        ("conv_pro", "s2 shortcut 256->512 s2 @87", 256, 87, 512, 1, 2, True, False),
        ("conv_pro", "s3 shortcut 512->1024 s2 @44", 512, 44, 1024, 1, 2, True, False),
        ("conv_glds", "s3 conv3 256->1024 +res @22", 256, 22, 1024, 1, 1, False, True),
        ("conv_glds", "s4 conv3 512->2048 +res @11", 512, 11, 2048, 1, 1, False, True),
        ("conv 3x3", "s3 conv2 3x3 256 @22", 256, 22, 256, 3, 1, False, False),
        ("conv 3x3", "s4 conv2 3x3 512 @11", 512, 11, 512, 3, 1, False, False),
    ]
    out = []
    g = torch.Generator(device="cpu").manual_seed(0)
    for fam, name, c, h, cout, ks, stride, pro, res in layers:
        x = torch.randn(b, c, h, h, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=CL)
        w = (torch.randn(cout, c, ks, ks, generator=g) * 0.05).to(dev, torch.bfloat16).contiguous(memory_format=CL)
        pad = ks // 2
        oh = (h + 2 * pad - ks) // stride + 1
        r = torch.randn(b, cout, oh, oh, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=CL) if res else None
        pr = (torch.rand(c, device=dev) + 0.5, torch.randn(c, device=dev) * 0.1) if pro else None
        t_nat = graph_us(lambda: C.conv2d(x, w, stride=stride, padding=pad, pro=pr, residual=r, act="none"))
        m, k = b * oh * oh, c * ks * ks
        a_ = torch.randn(m, k, generator=g).to(dev, torch.bfloat16)
        b_ = torch.randn(k, cout, generator=g).to(dev, torch.bfloat16)
        t_mm = graph_us(lambda: torch.mm(a_, b_))
        flop = 2.0 * m * k * cout
        byt = 2.0 * (b * h * h * c + m * cout * (2 if res else 1) + k * cout)
        out.append({"family": fam, "layer": name, "M": m, "K": k, "N": cout,
                    "native_us": round(t_nat, 1), "hipblaslt_us": round(t_mm, 1),
                    "native_vs_hipblaslt": round(t_mm / t_nat, 2),
                    "native_TBps": round(byt / t_nat / 1e6, 2), "native_TFLOPs": round(flop / t_nat / 1e6),
                    "hipblaslt_TFLOPs": round(flop / t_mm / 1e6)})
        print(json.dumps(out[-1]), flush=True)
    # conv23: stage-1/2 blocks' conv2 (3x3) + conv3 (1x1) + residual in one kernel,
    # against the two GEMMs it replaces
    from vgpu.models.resnet import FusedResNetV2Inference, resnet_v2_50
    model = resnet_v2_50().to(dev).to(torch.bfloat16).to(memory_format=CL).eval()
    fm = FusedResNetV2Inference(model)
    x = torch.randn(b, 3, 346, 346, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=CL)
    with torch.inference_mode():
        t_fwd = graph_us(lambda: fm(x), reps=3)
    for name, c, h in (("s1 conv2+conv3 64 @87", 64, 87), ("s2 conv2+conv3 128 @44", 128, 44)):
        m = b * h * h
        a2 = torch.randn(m, 9 * c, generator=g).to(dev, torch.bfloat16)
        b2 = torch.randn(9 * c, c, generator=g).to(dev, torch.bfloat16)
        a3 = torch.randn(m, c, generator=g).to(dev, torch.bfloat16)
        b3 = torch.randn(c, 4 * c, generator=g).to(dev, torch.bfloat16)
        t2 = graph_us(lambda: torch.mm(a2, b2))
        t3 = graph_us(lambda: torch.mm(a3, b3))
        out.append({"family": "conv23", "layer": name, "hipblaslt_two_gemms_us": round(t2 + t3, 1)})
        print(json.dumps(out[-1]), flush=True)
    print(json.dumps({"fused_forward_ms_b50": round(t_fwd / 1e3, 3)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
