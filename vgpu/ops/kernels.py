"""PyTorch-facing wrappers over the hand-written gfx950 kernels
(native/kernels/vgpu_kernels.hip, K1–K3 of SURVEY.md §2.9).

All functions run asynchronously on the current HIP stream and raise if the
native library is missing (no silent eager fallback).
"""
from __future__ import annotations

import ctypes

import torch

from vgpu.native import load_kernels


def _stream() -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with hipError {rc}")


def census(blocks: int, spin_ticks: int = 0) -> tuple[torch.Tensor, torch.Tensor]:
    """Launch `blocks` one-wave workgroups; returns (xcc_id, hw_id) int64 tensors
    of shape [blocks] and the spin ticks each workgroup measured."""
    out = torch.zeros(2 * blocks, dtype=torch.int32, device="cuda")
    ticks = torch.zeros(blocks, dtype=torch.int64, device="cuda")
    _check(load_kernels().vgpu_census(out.data_ptr(), blocks, spin_ticks, ticks.data_ptr(),
                                      _stream()), "vgpu_census")
    out = out.view(blocks, 2).to(torch.int64) & 0xFFFFFFFF
    return out, ticks


def decode_hw_id(hw_id: torch.Tensor) -> dict[str, torch.Tensor]:
    """gfx9 HW_ID fields: wave[3:0] simd[5:4] pipe[7:6] cu[11:8] sh[12] se[15:13]."""
    return {"cu": (hw_id >> 8) & 0xF, "sh": (hw_id >> 12) & 0x1, "se": (hw_id >> 13) & 0x7,
            "simd": (hw_id >> 4) & 0x3}


def busy(blocks: int, iters: int) -> None:
    sink = torch.empty(256, dtype=torch.float32, device="cuda")
    _check(load_kernels().vgpu_busy(sink.data_ptr(), blocks, iters, _stream()), "vgpu_busy")


def busy_via(blocks: int, iters: int, path: int) -> None:
    """busy() launched through hipLaunchKernel_spt (path 1) or a one-entry
    hipExtLaunchMultiKernelMultiDevice (path 2); 0 = hipLaunchKernel."""
    sink = torch.empty(256, dtype=torch.float32, device="cuda")
    _check(load_kernels().vgpu_busy_via(sink.data_ptr(), blocks, iters, _stream(), path), "vgpu_busy_via")


def gather_pages(dst: torch.Tensor, src: torch.Tensor, idx: torch.Tensor, page_bytes: int) -> None:
    """dst[k] = src[idx[k]] for pages of `page_bytes` (dst packed, src scattered)."""
    assert idx.dtype == torch.int64 and idx.is_cuda
    n = idx.numel()
    assert dst.numel() * dst.element_size() >= n * page_bytes
    if n:
        assert int(idx.max()) * page_bytes + page_bytes <= src.numel() * src.element_size()
    _check(load_kernels().vgpu_gather_pages(dst.data_ptr(), src.data_ptr(), idx.data_ptr(),
                                            page_bytes, n, _stream()), "vgpu_gather_pages")


def scatter_pages(dst: torch.Tensor, src: torch.Tensor, idx: torch.Tensor, page_bytes: int) -> None:
    """dst[idx[k]] = src[k]."""
    assert idx.dtype == torch.int64 and idx.is_cuda
    n = idx.numel()
    assert src.numel() * src.element_size() >= n * page_bytes
    if n:
        assert int(idx.max()) * page_bytes + page_bytes <= dst.numel() * dst.element_size()
    _check(load_kernels().vgpu_scatter_pages(dst.data_ptr(), src.data_ptr(), idx.data_ptr(),
                                             page_bytes, n, _stream()), "vgpu_scatter_pages")


def fill_pattern(t: torch.Tensor, seed: int) -> None:
    nbytes = t.numel() * t.element_size()
    _check(load_kernels().vgpu_fill_pattern(t.data_ptr(), nbytes - nbytes % 16, seed, _stream()),
           "vgpu_fill_pattern")


def verify_pattern(t: torch.Tensor, seed: int) -> int:
    nbytes = t.numel() * t.element_size()
    err = torch.zeros(1, dtype=torch.int64, device=t.device)
    _check(load_kernels().vgpu_verify_pattern(t.data_ptr(), nbytes - nbytes % 16, seed,
                                              err.data_ptr(), _stream()), "vgpu_verify_pattern")
    return int(err.item())


def pattern_reference(nbytes: int, seed: int) -> torch.Tensor:
    """CPU reference of the K3 fill (uint32 words), for numerics tests."""
    n = nbytes // 4
    i = torch.arange(n, dtype=torch.int64)
    # splitmix-style finalizer in 64-bit unsigned arithmetic emulated with int64 + masks
    M = (1 << 64) - 1
    vals = []
    for x in i.tolist():
        x = (x ^ ((seed * 0x9E3779B97F4A7C15) & M)) & M
        x ^= x >> 33
        x = (x * 0xff51afd7ed558ccd) & M
        x ^= x >> 33
        x = (x * 0xc4ceb9fe1a85ec53) & M
        x ^= x >> 33
        vals.append(x & 0xFFFFFFFF)
    return torch.tensor(vals, dtype=torch.int64)
