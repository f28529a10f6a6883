"""Fused stem conv + max pool vs the two-kernel path (ResNet stem at the
flagship shape, b=50 346²): per-call µs, in one process."""
import json
import torch
from vgpu.ops import conv as C
from vgpu.utils.timing import cuda_time_us

cl = torch.channels_last
x = torch.randn(50, 3, 346, 346, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)
w = C.stem_weight_s2d((torch.randn(64, 3, 7, 7, device="cuda") * (2 / 147) ** 0.5).to(torch.bfloat16))
two = lambda: C.maxpool3s2(C.stem_conv(x, w))  # noqa: E731
one = lambda: C.stem_pool(x, w)  # noqa: E731
s2d = lambda: C.stem_space_to_depth(x)  # noqa: E731
t = {"two_kernel_us": 0.0, "fused_us": 0.0, "s2d_only_us": 0.0}
for _ in range(3):
    t["two_kernel_us"] += cuda_time_us(two, 20) / 3
    t["fused_us"] += cuda_time_us(one, 20) / 3
    t["s2d_only_us"] += cuda_time_us(s2d, 20) / 3
print(json.dumps({k: round(v, 1) for k, v in t.items()} | {"bit_exact": bool(torch.equal(one(), two()))}))
