#!/usr/bin/env python3
"""In-process A/B of VGG-16's classifier at batch 2 (test 3.2): hipBLASLt
(F.linear + ReLU forward, autograd backward) against the skinny kernels
(vgpu.ops.linear), forward and forward+backward, each timed as a hipGraph
replay of 20 calls.  One JSON line per layer."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vgpu.utils.timing import graph_time_us as graph_us  # noqa: E402
from vgpu.ops.linear import _ACTS, _SkinnyLinearFn  # noqa: E402

torch.manual_seed(0)
for b, n, k, act in [(2, 4096, 25088, "relu"), (2, 4096, 4096, "relu"), (2, 1000, 4096, "none")]:
    x = torch.randn(b, k, device="cuda").to(torch.bfloat16).requires_grad_()
    w = (torch.randn(n, k, device="cuda") * k ** -0.5).to(torch.bfloat16).requires_grad_()
    bias = torch.zeros(n, device="cuda", dtype=torch.bfloat16).requires_grad_()
    dy = torch.randn(b, n, device="cuda").to(torch.bfloat16)

    def ref_fwd():
        y = F.linear(x, w, bias)
        return torch.relu(y) if act == "relu" else y

    def nat_fwd():
        return _SkinnyLinearFn.apply(x, w, bias, _ACTS[act])

    def step(f):
        def run():
            x.grad = w.grad = bias.grad = None
            f().backward(dy)
        return run

    res = {"layer": [b, n, k, act]}
    with torch.no_grad():
        res["fwd_blaslt_us"] = graph_us(ref_fwd)
        res["fwd_native_us"] = graph_us(nat_fwd)
    res["train_blaslt_us"] = graph_us(step(ref_fwd))
    res["train_native_us"] = graph_us(step(nat_fwd))
    res["weight_MB"] = round(n * k * 2 / 1e6, 1)
    print(json.dumps(res), flush=True)
