"""Prologue 1x1 convs: 128x256 tiles on 8 waves (conv_pro_kernel NT=512) against
128x128 on 4 waves, in one process, interleaved, at the flagship's layer shapes
with 128-row tiles forced (what a 50 % pod of the flagship picks)."""
import json
import torch
from vgpu.bench.convnative import layer_shapes
from vgpu.native import load_kernels
from vgpu.ops import conv as C
from vgpu.utils.timing import cuda_time_us

K = load_kernels()
cl = torch.channels_last
K.vgpu_conv_set_tile_m(128)
tot = [0.0, 0.0]
for name, n, c, h, w, cout, ks, stride, pad, ba, pro, res in layer_shapes(50, 346):
    if not pro or ks != 1 or cout % 256 or c < 192:
        continue
    x = torch.randn(n, c, h, w, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)
    wt = (torch.randn(cout, c, 1, 1, device="cuda") * (2 / c) ** 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
    b = torch.zeros(cout, device="cuda") if ba else None
    pp = (torch.rand(c, device="cuda") + 0.5, torch.randn(c, device="cuda") * 0.1)
    t = {0: 0.0, 1: 0.0}
    outs = {}
    for _ in range(3):
        for m in (1, 0):
            K.vgpu_conv_set_pro8(m)
            f = lambda: C.conv2d(x, wt, b, stride=stride, act="relu" if ba else "none", pro=pp)  # noqa: E731
            t[m] += cuda_time_us(f, 20) / 3
            outs[m] = f()
    tot[0] += t[1]
    tot[1] += t[0]
    print(json.dumps({"layer": name, "pro8_us": round(t[1], 1), "pro_us": round(t[0], 1),
                      "bit_exact": bool(torch.equal(outs[0], outs[1]))}), flush=True)
K.vgpu_conv_set_pro8(-1)
K.vgpu_conv_set_tile_m(0)
print(json.dumps({"total_pro8_us": round(tot[0], 1), "total_pro_us": round(tot[1], 1)}))
