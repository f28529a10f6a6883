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


def graph_time_us(fn: Callable[[], object], iters: int = 20, reps: int = 5) -> float:
    """Median µs per call of fn replayed from a hipGraph of `iters` calls
    (host launch overhead excluded: the training steps are graph replays)."""
    import torch
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    times = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1) * 1e3 / iters)
    return round(sorted(times)[len(times) // 2], 2)
