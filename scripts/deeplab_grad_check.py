#!/usr/bin/env python3
"""DeepLab-v3 training-step gradients: native bf16, PyTorch/MIOpen bf16 and
PyTorch fp32 from the same weights, padded (pad_channels=64) and unpadded;
cosine of depthwise / stem / head weight gradients against fp32.

    python scripts/deeplab_grad_check.py [--hw 64] [--batch 2]
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CL = torch.channels_last


def cos(a, b):
    return round(torch.nn.functional.cosine_similarity(a.float().flatten(), b.float().flatten(), dim=0).item(), 4)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--hw", type=int, default=64)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--classes", type=int, default=5)
    a = ap.parse_args()
    from vgpu.models.vision import DeepLabV3
    from vgpu.ops import conv as C
    for pad in (1, 64):
        torch.manual_seed(0)
        base = DeepLabV3(num_classes=a.classes, pad_channels=pad).cuda().train()
        g = torch.Generator().manual_seed(7)
        x = torch.randn(a.batch, 3, a.hw, a.hw, generator=g).cuda()
        tgt = torch.randint(0, a.classes, (a.batch, a.hw, a.hw), device="cuda")
        runs = {}
        for name, dt, native in (("fp32", torch.float32, False), ("torch_bf16", torch.bfloat16, False),
                                 ("native_bf16", torch.bfloat16, True)):
            m = copy.deepcopy(base).to(dt).to(memory_format=CL)
            C._TRAIN_NATIVE = native
            try:
                out = m(x.to(dt).contiguous(memory_format=CL))
                loss = torch.nn.functional.cross_entropy(out.float(), tgt)
                loss.backward()
            finally:
                C._TRAIN_NATIVE = True
            grads = {"stem": m.backbone.features[0][0].weight.grad, "head": m.head.weight.grad}
            for i in (1, 5, 12, 16):
                grads[f"dw{i}"] = m.backbone.features[i].body[-2][0].weight.grad
            runs[name] = (loss.item(), grads)
        ref_loss, ref = runs["fp32"]
        for name in ("torch_bf16", "native_bf16"):
            loss, gr = runs[name]
            print(json.dumps({"pad": pad, "path": name, "loss": round(loss, 5), "loss_fp32": round(ref_loss, 5),
                              **{k: cos(v, ref[k]) for k, v in gr.items()}}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
