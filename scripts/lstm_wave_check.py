#!/usr/bin/env python3
"""Intermediate tensors of the two-layer wavefront LSTM against the
layer-by-layer path on the same inputs (debug aid for vgpu.ops.lstm):
layer-1 h, layer 2's projection, layer-2 h / gates / cells, and the backward's
dgates and layer-1 output gradient."""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rel(a, b):
    a, b = a.float(), b.float()
    return round(float((a - b).abs().max() / (b.abs().max() + 1e-9)), 5)


def main() -> int:
    from vgpu.native import load_kernels
    from vgpu.ops import lstm as L
    lib = load_kernels()
    torch.manual_seed(1)
    b, t, e, h = int(sys.argv[1]) if len(sys.argv) > 1 else 10, 40, 300, 128
    mod = torch.nn.LSTM(e, h, num_layers=2, batch_first=True).cuda().to(torch.bfloat16)
    x = (torch.randn(b, t, e, device="cuda") * 0.5).to(torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream
    # layer by layer
    xt = x.transpose(0, 1).reshape(t * b, -1)
    xp1 = torch.addmm(mod.bias_ih_l0 + mod.bias_hh_l0, xt, mod.weight_ih_l0.t()).view(t, b, 4 * h)
    y1 = torch.empty(b, t, h, dtype=x.dtype, device="cuda")
    g1 = torch.empty(t, b, 4 * h, dtype=x.dtype, device="cuda")
    c1 = torch.empty(t, b, h, dtype=torch.float32, device="cuda")
    assert lib.vgpu_lstm_forward_train(xp1.data_ptr(), mod.weight_hh_l0.contiguous().data_ptr(), y1.data_ptr(),
                                       g1.data_ptr(), c1.data_ptr(), b, t, h, st) == 0
    xp2_ref = torch.addmm(mod.bias_ih_l1 + mod.bias_hh_l1, y1.transpose(0, 1).reshape(t * b, h),
                          mod.weight_ih_l1.t()).view(t, b, 4 * h)
    y2 = torch.empty(b, t, h, dtype=x.dtype, device="cuda")
    g2 = torch.empty_like(g1)
    c2 = torch.empty_like(c1)
    assert lib.vgpu_lstm_forward_train(xp2_ref.data_ptr(), mod.weight_hh_l1.contiguous().data_ptr(), y2.data_ptr(),
                                       g2.data_ptr(), c2.data_ptr(), b, t, h, st) == 0
    # wavefront
    y1t = torch.empty(t, b, h, dtype=x.dtype, device="cuda")
    y2t = torch.empty_like(y1t)
    xp2 = torch.empty(t, b, 4 * h, dtype=x.dtype, device="cuda")
    wg1, wg2 = torch.empty_like(g1), torch.empty_like(g1)
    wc1, wc2 = torch.empty_like(c1), torch.empty_like(c1)
    flags = L._flags(b, "cuda")
    b2 = (mod.bias_ih_l1 + mod.bias_hh_l1).contiguous()
    assert lib.vgpu_lstm2_forward(xp1.data_ptr(), mod.weight_hh_l0.contiguous().data_ptr(),
                                  mod.weight_ih_l1.contiguous().data_ptr(), b2.data_ptr(),
                                  mod.weight_hh_l1.contiguous().data_ptr(), y1t.data_ptr(), xp2.data_ptr(),
                                  flags.data_ptr(), None, y2t.data_ptr(), wg1.data_ptr(), wg2.data_ptr(),
                                  wc1.data_ptr(), wc2.data_ptr(), b, t, h, st) == 0
    torch.cuda.synchronize()
    print("error flag", lib.vgpu_lstm2_flags_error(flags.data_ptr(), b))
    print("fwd: y1", rel(y1t, y1.transpose(0, 1)), "xp2", rel(xp2, xp2_ref), "y2", rel(y2t, y2.transpose(0, 1)),
          "gates1", rel(wg1, g1), "gates2", rel(wg2, g2), "cells2", rel(wc2, c2))
    for tt in (0, 1, 2, t - 1):
        print("  xp2 step", tt, rel(xp2[tt], xp2_ref[tt]), "y1 step", rel(y1t[tt], y1[:, tt]))
    # backward on identical saved state (the layered one)
    dy2 = torch.zeros(b, t, h, dtype=x.dtype, device="cuda")
    dy2[:, -1] = (torch.randn(b, h, device="cuda")).to(x.dtype)
    dg2 = torch.empty_like(g1)
    assert lib.vgpu_lstm_backward(g2.data_ptr(), c2.data_ptr(), dy2.data_ptr(), mod.weight_hh_l1.contiguous().data_ptr(),
                                  dg2.data_ptr(), b, t, h, st) == 0
    dy1_ref = (dg2.view(t * b, 4 * h) @ mod.weight_ih_l1).view(t, b, h)
    dg1 = torch.empty_like(g1)
    assert lib.vgpu_lstm_backward(g1.data_ptr(), c1.data_ptr(), dy1_ref.transpose(0, 1).contiguous().data_ptr(),
                                  mod.weight_hh_l0.contiguous().data_ptr(), dg1.data_ptr(), b, t, h, st) == 0
    wdg1, wdg2, wdy1 = torch.empty_like(g1), torch.empty_like(g1), torch.empty_like(y1t)
    assert lib.vgpu_lstm2_backward(g1.data_ptr(), c1.data_ptr(), g2.data_ptr(), c2.data_ptr(), dy2.data_ptr(),
                                   mod.weight_hh_l0.contiguous().data_ptr(), mod.weight_hh_l1.contiguous().data_ptr(),
                                   mod.weight_ih_l1.contiguous().data_ptr(), wdg1.data_ptr(), wdg2.data_ptr(),
                                   wdy1.data_ptr(), flags.data_ptr(), b, t, h, st) == 0
    torch.cuda.synchronize()
    print("error flag", lib.vgpu_lstm2_flags_error(flags.data_ptr(), b))
    print("bwd: dgates2", rel(wdg2, dg2), "dy1", rel(wdy1, dy1_ref), "dgates1", rel(wdg1, dg1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
