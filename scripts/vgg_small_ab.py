#!/usr/bin/env python3
"""In-process A/B for VGG-16 training at batch 2 (ai-benchmark test 3.2): the
convs whose output tiles cannot fill the GPU (28² / 14² / 56² layers) with
and without split-K, and three weight-gradient routes for them (MIOpen's
convolution_backward, the native wgrad kernel, im2col + hipBLASLt GEMM).
Every variant is captured in a hipGraph of `iters` calls and replayed, so host
launch overhead is excluded (the training step itself is a graph replay).

    python scripts/vgg_small_ab.py            -> one JSON line per shape
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vgpu.ops import conv as C  # noqa: E402
from vgpu.utils.timing import graph_time_us  # noqa: E402

CL = torch.channels_last


graph_us = graph_time_us


def wgrad_gemm(dy, x, ks=3, pad=1):
    n, c, h, w = x.shape
    cout, oh, ow = dy.shape[1:]
    xp = F.pad(x.permute(0, 2, 3, 1), (0, 0, pad, pad, pad, pad))
    cols = torch.stack([xp[:, kh:kh + oh, kw:kw + ow, :] for kh in range(ks) for kw in range(ks)], dim=3)
    dw = dy.permute(0, 2, 3, 1).reshape(-1, cout).t() @ cols.reshape(n * oh * ow, ks * ks * c)
    return dw.view(cout, ks, ks, c).permute(0, 3, 1, 2)


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


torch.manual_seed(0)
SHAPES = [(2, 256, 56, 256), (2, 256, 28, 512), (2, 512, 28, 512), (2, 512, 14, 512),
          # ResNet-V2-152 b=10 stages 3 / 4, ResNet-V2-50 training stage 4 (tests 2.2 / 1.2)
          (10, 256, 16, 256), (10, 512, 8, 512), (50, 512, 7, 512)]
if len(sys.argv) > 1:
    SHAPES = [SHAPES[int(i)] for i in sys.argv[1:]]
for n, c, hw, cout in SHAPES:
    x = torch.randn(n, c, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(cout, c, 3, 3, device="cuda") * (2 / (9 * c)) ** 0.5).to(torch.bfloat16).contiguous(memory_format=CL)
    b = torch.randn(cout, device="cuda").to(torch.bfloat16)
    dy = torch.randn(n, cout, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    res = {"shape": [n, c, hw, cout]}
    C.set_splitk(0)
    y0 = C.conv2d(x, w, b, padding=1, act="relu")
    res["fwd_unsplit_us"] = graph_us(lambda: C.conv2d(x, w, b, padding=1, act="relu"))
    C.set_splitk(-1)
    y1 = C.conv2d(x, w, b, padding=1, act="relu")
    res["fwd_split_us"] = graph_us(lambda: C.conv2d(x, w, b, padding=1, act="relu"))
    res["fwd_split_rel"] = round(rel(y1, y0), 5)
    ref = F.relu(F.conv2d(x.float(), w.float(), b.float(), padding=1))
    res["fwd_split_rel_fp32"] = round(rel(y1, ref), 5)
    common = ([0], [1, 1], [1, 1], [1, 1], False, [0, 0], 1)
    bw = torch.ops.aten.convolution_backward
    d0 = bw(dy, x, w, *common, [False, True, False])[1]
    d1 = C.conv2d_wgrad(dy, x, 3, padding=1)
    d2 = wgrad_gemm(dy, x)
    res["wgrad_miopen_us"] = graph_us(lambda: bw(dy, x, w, *common, [False, True, False]))
    res["wgrad_native_us"] = graph_us(lambda: C.conv2d_wgrad(dy, x, 3, padding=1))
    res["wgrad_gemm_us"] = graph_us(lambda: wgrad_gemm(dy, x))
    res["wgrad_native_rel"] = round(rel(d1, d0), 5)
    res["wgrad_gemm_rel"] = round(rel(d2, d0), 5)
    print(json.dumps(res), flush=True)
