#!/usr/bin/env python3
"""Speed-of-light of the flagship step: the kernel plan of the native ResNet-V2
inference forward (vgpu/models/resnet.py `_forward_native`), each kernel's
compulsory HBM bytes (inputs once, weights once, outputs once) and MFMA FLOPs,
and the time it cannot beat on one MI355X (8 TB/s HBM3E, 2.5 PFLOP/s dense bf16).

    python scripts/roofline.py [--batch 50] [--size 346] [--pods 2] [--measured-ms 3.90]

CPU only: the plan is derived from the model's layer shapes, mirroring the
dispatch decisions of `_forward_native` (conv23/conv231 fusion for C in
{64, 128}; separate conv2/conv3 otherwise).  `--measured-ms` is the bench's
ms_per_step (all pods) to compare against.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HBM_TBPS = 8.0
MFMA_PFLOPS = 2.5
E = 2  # bf16 bytes


def plan(batch: int, size: int, layers=(3, 4, 6, 3)):
    """[(kernel, flops, bytes)] of one forward at (batch, 3, size, size)."""
    out = []

    def conv_out(h, k, s, p):
        return (h + 2 * p - k) // s + 1

    # stem: 7x7/s2/p3 conv 3->64 as space-to-depth + 4x4 conv, with the 3x3/s2
    # max-pool fused (conv_gemm.hip stem_pool_kernel): the stem activation stays
    # on chip (model FLOPs counted; the kernel recomputes one stem row in three)
    h = conv_out(size, 7, 2, 3)
    m = batch * h * h
    h2 = conv_out(h, 3, 2, 1)
    hs = h + 3
    out.append(("stem conv + maxpool", 2 * m * 7 * 7 * 3 * 64,
                E * (batch * size * size * 3 + batch * hs * hs * 16 * 2 + batch * h2 * h2 * 64 + 7 * 7 * 3 * 64)))
    h = h2
    cin = 64
    blocks = []
    for st, n in enumerate(layers):
        width = 64 << st
        for i in range(n):
            stride = 2 if (i == 0 and st > 0) else 1
            blocks.append((cin, width, stride, i == 0))
            cin = width * 4
    h_next_ready = False
    for bi, (ci, wd, stride, proj) in enumerate(blocks):
        co = wd * 4
        m_in = batch * h * h
        ho = conv_out(h, 3, stride, 1)
        m_out = batch * ho * ho
        if proj:
            out.append((f"b{bi} shortcut 1x1 (BN+ReLU prologue)", 2 * m_out * ci * co,
                        E * (m_in * ci + m_out * co + ci * co)))
        if not h_next_ready:
            out.append((f"b{bi} conv1 1x1 (BN+ReLU prologue)", 2 * m_in * ci * wd, E * (m_in * ci + m_in * wd + ci * wd)))
        h_next_ready = False
        nxt = blocks[bi + 1] if bi + 1 < len(blocks) else None
        f2 = 2 * m_out * 9 * wd * wd
        f3 = 2 * m_out * wd * co
        w23 = E * (9 * wd * wd + wd * co)
        if wd in (64, 128) and nxt is not None and not nxt[3]:
            f1n = 2 * m_out * co * nxt[1]
            out.append((f"b{bi} conv2+conv3+res+next conv1", f2 + f3 + f1n,
                        E * (m_in * wd + m_out * co * 2 + m_out * nxt[1] + co * nxt[1]) + w23))
            h_next_ready = True
        elif wd in (64, 128):
            out.append((f"b{bi} conv2+conv3+res", f2 + f3, E * (m_in * wd + m_out * co * 2) + w23))
        else:
            out.append((f"b{bi} conv2 3x3", f2, E * (m_in * wd + m_out * wd + 9 * wd * wd)))
            out.append((f"b{bi} conv3 1x1 + res", f3, E * (m_out * wd + 2 * m_out * co + wd * co)))
        h = ho
    out.append(("BN+ReLU+mean", 0, E * batch * h * h * cin))
    out.append(("fc", 2 * batch * cin * 1000, E * (cin * 1000 + batch * cin)))
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=50)
    ap.add_argument("--size", type=int, default=346)
    ap.add_argument("--pods", type=int, default=2)
    ap.add_argument("--measured-ms", type=float, default=None, help="bench ms_per_step (all pods)")
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args(argv)
    ks = plan(a.batch, a.size)
    fl = sum(k[1] for k in ks)
    by = sum(k[2] for k in ks)
    # per kernel the bound is max(bytes, flops); the step bound sums them
    t_k = sum(max(b / (HBM_TBPS * 1e12), f / (MFMA_PFLOPS * 1e15)) for _, f, b in ks) * 1e3
    res = {"batch": a.batch, "size": a.size, "pods": a.pods, "kernels": len(ks),
           "gflop_per_image": round(fl / a.batch / 1e9, 2), "hbm_gb_per_forward": round(by / 1e9, 3),
           "bound_ms_per_forward_bytes": round(by / (HBM_TBPS * 1e12) * 1e3, 3),
           "bound_ms_per_forward_flops": round(fl / (MFMA_PFLOPS * 1e15) * 1e3, 3),
           "bound_ms_per_forward_sum_of_kernel_max": round(t_k, 3)}
    step_bound = t_k * a.pods
    res["bound_ms_per_step"] = round(step_bound, 3)
    res["bound_images_s"] = round(a.batch * a.pods / step_bound * 1e3, 0)
    if a.measured_ms:
        res["measured_ms_per_step"] = a.measured_ms
        res["fraction_of_speed_of_light"] = round(step_bound / a.measured_ms, 3)
        res["achieved_tflops"] = round(fl * a.pods / (a.measured_ms * 1e-3) / 1e12, 1)
    if a.json:
        print(json.dumps(res))
        return 0
    print("| kernel | GFLOP | MB | bound us | bound by |\n|---|---|---|---|---|")
    for name, f, b in ks:
        tb, tf = b / (HBM_TBPS * 1e12) * 1e6, f / (MFMA_PFLOPS * 1e15) * 1e6
        print(f"| {name} | {f / 1e9:.1f} | {b / 1e6:.1f} | {max(tb, tf):.1f} | {'HBM' if tb >= tf else 'MFMA'} |")
    print()
    print(json.dumps(res, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
