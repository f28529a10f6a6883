"""Per-layer timing of the training-time convolution passes of ResNet-V2-50
(ai-benchmark test 1.2: b=20, 346²): MIOpen forward / backward-data /
backward-weight against the native candidates.

    python scripts/convtrain.py [--batch 20 --size 346 --iters 20]

Native candidates per layer (stride-1 only for the data gradient):
  fwd    native MFMA implicit GEMM (vgpu.ops.conv.conv2d)
  dgrad  the same kernel on dy with the transposed (and, for 3x3, flipped) filter
  wgrad  native MFMA weight gradient (vgpu.ops.conv.conv2d_wgrad: transposed LDS
         reads, split-K over pixels); the earlier 1x1-as-hipBLASLt-GEMM candidate
         (dW = dyᵀ·x) measured 3.4x slower than MIOpen (profiles/convtrain_r1.md)
One JSON line per layer plus a total line.
"""
from __future__ import annotations

import os as _os
import sys as _sys

_here = _os.path.dirname(_os.path.abspath(__file__))
_sys.path[:0] = [_here, _os.path.dirname(_here)]  # scripts/ and the repo root

import argparse
import json

from convnative import layer_shapes  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=20)
    ap.add_argument("--size", type=int, default=346)
    ap.add_argument("--iters", type=int, default=20)
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

    tot = {}
    for name, n, c, h, w, cout, ks, stride, pad, _ba, _pro, _res in layer_shapes(args.batch, args.size):
        x = torch.randn(n, c, h, w, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        wt = (torch.randn(cout, c, ks, ks, device=dev) * (2 / (c * ks * ks)) ** 0.5).to(
            torch.bfloat16).contiguous(memory_format=cl)
        oh, ow = C.out_hw(h, w, ks, stride, pad)
        dy = torch.randn(n, cout, oh, ow, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        bw = torch.ops.aten.convolution_backward
        common = ([0], [stride, stride], [pad, pad], [1, 1], False, [0, 0], 1)
        r = {"layer": name, "M": n * oh * ow, "C": c, "Cout": cout, "ks": ks, "stride": stride}
        r["mio_fwd"] = timeit(lambda: F.conv2d(x, wt, stride=stride, padding=pad))
        r["mio_dgrad"] = timeit(lambda: bw(dy, x, wt, *common, [True, False, False]))
        r["mio_wgrad"] = timeit(lambda: bw(dy, x, wt, *common, [False, True, False]))
        r["mio_both"] = timeit(lambda: bw(dy, x, wt, *common, [True, True, False]))
        r["nat_fwd"] = timeit(lambda: C.conv2d(x, wt, stride=stride, padding=pad))
        if stride == 1 and cout % 64 == 0 and c % 64 == 0:
            wt_t = wt.permute(1, 0, 2, 3).flip(2, 3).contiguous(memory_format=cl)
            r["nat_dgrad"] = timeit(lambda: C.conv2d(dy, wt_t, stride=1, padding=ks - 1 - pad))
            ref = bw(dy, x, wt, *common, [True, False, False])[0]
            got = C.conv2d(dy, wt_t, stride=1, padding=ks - 1 - pad)
            r["dgrad_err"] = ((got.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
        r["nat_wgrad"] = timeit(lambda: C.conv2d_wgrad(dy, x, ks, stride=stride, padding=pad))
        ref = bw(dy, x, wt, *common, [False, True, False])[1]
        got = C.conv2d_wgrad(dy, x, ks, stride=stride, padding=pad)
        r["wgrad_err"] = ((got.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
        for k, v in list(r.items()):
            if k.startswith(("mio_", "nat_")):
                r[k] = round(v, 1)
                tot[k] = tot.get(k, 0.0) + v
        print(json.dumps(r), flush=True)
    print(json.dumps({"total_us": {k: round(v, 1) for k, v in tot.items()}}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
