"""GPU timing helpers shared by the per-kernel benchmarks (convnative,
convtrain, convab, gemm_ceiling): HIP-event timing of a callable, and an
in-process interleaved A/B (box-to-box variance on this pool is ±10 % per
kernel, so variants are compared in one process, alternating)."""
from __future__ import annotations

from typing import Callable, Sequence


def cuda_time_us(fn: Callable[[], object], iters: int = 20, warmup: int = 3) -> float:
    """Mean µs per call of fn on the current stream (HIP events around `iters` calls)."""
    import torch
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def interleaved_us(fns: Sequence[Callable[[], object]], rounds: int = 3, iters: int = 20) -> list[float]:
    """Mean µs per call of each fn, measured round-robin `rounds` times."""
    tot = [0.0] * len(fns)
    for _ in range(rounds):
        for i, fn in enumerate(fns):
            tot[i] += cuda_time_us(fn, iters) / rounds
    return tot
