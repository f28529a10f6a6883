#!/usr/bin/env python3
"""LSTM recurrence on MI355X: where a timestep's time goes, and what the
two-layer wavefront buys.

1. Phase profile: one layer's recurrence (B rows, T steps) with s_memtime
   stamps in workgroup 0 (native/kernels/lstm.hip, FwdArgs::prof): cycles per
   step in (0) Xp wait + h read, (1) MFMA + gate activations + cell update
   (in registers), (3) h / output stores, (4) the step's barrier.  The stamps themselves serialise the wave a little; the plain
   kernel's time per step is reported next to it.
2. 5.1 / 5.2 shapes end to end: layer by layer (VGPU_LSTM_WAVE=0) against the
   wavefront launch, inference (B=100) and a training step (B=10).

    python scripts/lstm_profile.py > profiles/r6/lstm/lstm_profile.json
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def phase_profile(b=100, t=1024, h=128):
    from vgpu.native import load_kernels
    lib = load_kernels()
    dev = "cuda"
    xp = (torch.randn(t, b, 4 * h, device=dev) * 0.5).to(torch.bfloat16)
    whh = (torch.randn(4 * h, h, device=dev) * 0.05).to(torch.bfloat16)
    y = torch.empty(t, b, h, dtype=torch.bfloat16, device=dev)
    hs = torch.empty(b, h, dtype=torch.bfloat16, device=dev)
    cs = torch.empty(b, h, dtype=torch.float32, device=dev)
    prof = torch.zeros(8, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream().cuda_stream

    def run(p):
        rc = lib.vgpu_lstm_recurrence_window(xp.data_ptr(), whh.data_ptr(), y.data_ptr(), h, b * h, hs.data_ptr(),
                                             cs.data_ptr(), 1, None, None, b, t, h, p, st)
        assert rc == 0, rc

    plain_ms = timed(lambda: run(None))
    prof_ms = timed(lambda: run(prof.data_ptr()), reps=3, warm=1)
    cyc = prof[:5].double().cpu() / t
    total = float(cyc.sum())
    names = ["xp_wait_and_h_read", "mfma_activations_and_cell_update", "unused", "h_and_output_stores", "barrier"]
    return {"B": b, "T": t, "plain_us_per_step": round(plain_ms * 1e3 / t, 3),
            "profiled_us_per_step": round(prof_ms * 1e3 / t, 3),
            "cycles_per_step": round(total, 1),
            "clock_GHz_implied": round(total / (prof_ms * 1e6 / t), 3),
            "phases": {n: {"cycles": round(float(c), 1), "share": round(float(c) / total, 3)}
                       for n, c in zip(names, cyc)}}


def end_to_end():
    from vgpu.models.vision import LSTMSentiment
    out = {}
    for name, b, train in (("5.1 inference b=100", 100, False), ("5.2 training b=10", 10, True)):
        torch.manual_seed(0)
        m = LSTMSentiment().cuda().to(torch.bfloat16)
        x = (torch.randn(b, 1024, 300, device="cuda") * 0.5).to(torch.bfloat16)
        tgt = torch.randint(0, 2, (b,), device="cuda")
        row = {}
        for mode in ("0", "1"):
            os.environ["VGPU_LSTM_WAVE"] = mode
            if train:
                m.train()

                def step():
                    m.zero_grad(set_to_none=True)
                    torch.nn.functional.cross_entropy(m(x).float(), tgt).backward()
            else:
                m.eval()

                def step():
                    with torch.no_grad():
                        m(x)
            ms = timed(step, reps=10)
            row["wavefront" if mode == "1" else "layer_by_layer"] = {"ms": round(ms, 3),
                                                                     "seq_per_s": round(b / ms * 1e3, 1)}
        row["speedup"] = round(row["layer_by_layer"]["ms"] / row["wavefront"]["ms"], 3)
        out[name] = row
    os.environ.pop("VGPU_LSTM_WAVE", None)
    return out


def main() -> int:
    res = {"phase_profile_b100": phase_profile(100), "phase_profile_b10": phase_profile(10),
           "end_to_end": end_to_end()}
    print(json.dumps(res, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
