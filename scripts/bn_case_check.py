#!/usr/bin/env python3
"""One BatchNorm test case split in two: the PyTorch fp32 reference alone
(`ref`), or the native forward + backward alone (`native`).

    python scripts/bn_case_check.py ref|native N C H W OFFSET
"""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))


def main() -> int:
    which = sys.argv[1]
    n, c, h, w = map(int, sys.argv[2:6])
    off = float(sys.argv[6])
    g = torch.Generator(device="cpu").manual_seed(1)
    x = (torch.randn((n, c, h, w), generator=g) + off).to(torch.bfloat16).cuda().contiguous(
        memory_format=torch.channels_last)
    wt = torch.rand(c).cuda() + 0.5
    bs = torch.rand(c).cuda() - 0.5
    rm, rv = torch.zeros(c).cuda(), torch.ones(c).cuda()
    if which == "ref":
        from vgpu.ops import bn as B
        y = B.bn_act_reference(x.float().requires_grad_(), wt, bs, rm, rv, 0.1, 1e-5, "relu6")
    else:
        from vgpu.ops import bn as B
        xr = x.clone().requires_grad_()
        y = B._BNActFn.apply(xr, wt.clone().requires_grad_(), bs.clone().requires_grad_(), rm, rv, 0.1, 1e-5,
                             B.ACT["relu6"])
        y.backward(torch.ones_like(y))
    torch.cuda.synchronize()
    print(which, "ok", float(y.float().sum()), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
