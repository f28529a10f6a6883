#!/usr/bin/env python3
"""In-process A/B of the fused stem conv + max pool: the tree's
libvgpu_kernels.so against another build of vgpu_stem_pool_nhwc given on the
command line (e.g. an older conv_gemm.hip compiled alone into build_ab/).
Interleaved timing on the ResNet-50 flagship shape (b=50, 346²), outputs
compared bit for bit.

    python scripts/stem_lib_ab.py build_ab/libstem_old.so [batch] [reps]
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vgpu.native import load_kernels  # noqa: E402
from vgpu.ops import conv as C  # noqa: E402

other = ctypes.CDLL(os.path.abspath(sys.argv[1]))
B = int(sys.argv[2]) if len(sys.argv) > 2 else 50
REPS = int(sys.argv[3]) if len(sys.argv) > 3 else 20
vp, ci = ctypes.c_void_p, ctypes.c_int
other.vgpu_stem_pool_nhwc.argtypes = [vp, vp, vp] + [ci] * 3 + [vp]
other.vgpu_stem_pool_nhwc.restype = ci
cur = load_kernels()

torch.manual_seed(0)
x = torch.randn(B, 3, 346, 346, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
w = C.stem_weight_s2d((torch.randn(64, 3, 7, 7, device="cuda") * 0.1).to(torch.bfloat16))
X = C.stem_space_to_depth(x)
n, _, hs, ws = X.shape
ref = C.stem_pool(x, w)
outs = {k: torch.empty_like(ref) for k in ("cur", "other")}
libs = {"cur": cur, "other": other}
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def run(k):
    rc = libs[k].vgpu_stem_pool_nhwc(vp(X.data_ptr()), vp(w.data_ptr()), vp(outs[k].data_ptr()), n, hs, ws, s)
    assert rc == 0, (k, rc)


times = {k: [] for k in libs}
for k in libs:
    run(k)
torch.cuda.synchronize()
for r in range(REPS):
    for k in (("cur", "other") if r % 2 == 0 else ("other", "cur")):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            run(k)
        e1.record()
        torch.cuda.synchronize()
        times[k].append(e0.elapsed_time(e1) * 100)  # us per launch
res = {k: round(sorted(v)[len(v) // 2], 1) for k, v in times.items()}
res["bit_identical"] = bool(torch.equal(outs["cur"], outs["other"]) and torch.equal(outs["cur"], ref))
res["batch"] = B
print(json.dumps(res))
