"""Bilinear resize (align_corners=False) whose backward is two small GEMMs.

PyTorch's bilinear-upsample backward scatters every output gradient into its
four source pixels with atomic adds; for DeepLab-v3's 24² → 384² logit
upsample (and the ASPP image-pool broadcast, 1² → 24²) that is ~256 bf16
atomics per source element, serialised CAS loops: 4.3 ms per dispatch, 71 % of
the 4.2 training step (profiles/r5/train/prof_4_2_before.md).  The resize is
separable and linear, y = A_h · x · A_wᵀ per (n, c), with A_h [OH, IH] and A_w
[OW, IW] holding PyTorch's two interpolation weights per row, so
dx = A_hᵀ · dy · A_w: two batched fp32 GEMMs (hipBLASLt), no atomics,
deterministic.  The forward is PyTorch's gather kernel; with
VGPU_NATIVE_RESIZE=1 bf16 channels-last tensors run on
native/kernels/resize.hip instead (one thread per output pixel; PyTorch's NHWC
kernel took 26 us per 4.1 logit upsample).
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.nn.functional as F

_MATS: dict[tuple, torch.Tensor] = {}
# VGPU_NATIVE_RESIZE=1: the native forward (not yet measured on MI355X end to end, so off by default)
_NATIVE = os.environ.get("VGPU_NATIVE_RESIZE", "0") == "1"
_BOUND = False


def _forward(x: torch.Tensor, size, native: bool | None = None) -> torch.Tensor:
    """F.interpolate(x, size, bilinear, align_corners=False); native for bf16
    channels-last CUDA tensors when enabled (native=None: VGPU_NATIVE_RESIZE)."""
    if not ((_NATIVE if native is None else native) and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4
            and x.is_contiguous(memory_format=torch.channels_last)):
        return F.interpolate(x, size=size, mode="bilinear", align_corners=False)
    global _BOUND
    from vgpu.native import load_kernels
    lib = load_kernels()
    if not _BOUND:
        vp, ci = ctypes.c_void_p, ctypes.c_int
        lib.vgpu_resize_bilinear_nhwc.argtypes = [vp, vp] + [ci] * 6 + [vp]
        lib.vgpu_resize_bilinear_nhwc.restype = ci
        _BOUND = True
    n, c, ih, iw = x.shape
    oh, ow = size
    y = torch.empty((n, c, oh, ow), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
    rc = lib.vgpu_resize_bilinear_nhwc(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()), n, ih, iw, c,
                                       oh, ow, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    if rc != 0:
        raise RuntimeError(f"vgpu_resize_bilinear_nhwc: error {rc}")
    return y


def interp_matrix(out: int, inp: int, device) -> torch.Tensor:
    """[out, inp] fp32: row o holds PyTorch's bilinear (align_corners=False)
    weights of output o: src = max((o + 0.5)·inp/out - 0.5, 0), i0 = ⌊src⌋,
    i1 = min(i0 + 1, inp - 1), weights 1 - λ and λ = src - i0."""
    key = (out, inp, str(device))
    m = _MATS.get(key)
    if m is None:
        o = torch.arange(out, dtype=torch.float64)
        src = ((o + 0.5) * (inp / out) - 0.5).clamp_min(0.0)
        i0 = src.floor().long().clamp_max(inp - 1)
        i1 = torch.where(i0 < inp - 1, i0 + 1, i0)
        lam = (src - i0.double()).clamp(0.0, 1.0)
        m = torch.zeros(out, inp, dtype=torch.float64)
        m.index_put_((torch.arange(out), i0), 1.0 - lam, accumulate=True)
        m.index_put_((torch.arange(out), i1), lam, accumulate=True)
        m = m.to(torch.float32).to(device)
        _MATS[key] = m
    return m


class _ResizeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, size):
        ctx.in_hw = tuple(x.shape[-2:])
        ctx.cl = x.is_contiguous(memory_format=torch.channels_last)
        return _forward(x, size)

    @staticmethod
    def backward(ctx, dy):
        (ih, iw), (oh, ow) = ctx.in_hw, tuple(dy.shape[-2:])
        ah = interp_matrix(oh, ih, dy.device)
        aw = interp_matrix(ow, iw, dy.device)
        g = torch.matmul(torch.matmul(ah.t(), dy.float()), aw)  # [N, C, IH, IW]
        g = g.to(dy.dtype)
        return (g.contiguous(memory_format=torch.channels_last) if ctx.cl else g.contiguous()), None


def resize_bilinear(x: torch.Tensor, size) -> torch.Tensor:
    """F.interpolate(x, size, mode="bilinear", align_corners=False) with the
    GEMM backward on CUDA tensors that need a gradient; PyTorch's otherwise."""
    size = tuple(int(s) for s in size)
    if not (x.is_cuda and x.requires_grad and torch.is_grad_enabled() and x.dim() == 4):
        return _forward(x, size) if x.dim() == 4 else F.interpolate(x, size=size, mode="bilinear",
                                                                     align_corners=False)
    return _ResizeFn.apply(x, size)
