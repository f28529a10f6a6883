"""Mean cross-entropy over logits with integer targets on one native kernel
pass (native/kernels/loss.hip): the forward also writes the gradient, so the
backward is a single scale by the incoming gradient.  Same value and
gradient as torch.nn.functional.cross_entropy(logits.float(), target,
ignore_index=...) with reduction 'mean' (no class weights, no label
smoothing), for

* classification logits [rows, C] and targets [rows];
* per-pixel logits [B, C, H, W] (NCHW or channels-last, read in place) and
  targets [B, H, W] -- DeepLab's loss, PyTorch's nll_loss2d path.

A target outside [0, C) or equal to ``ignore_index`` drops its row from the
loss and the mean, as PyTorch's ``ignore_index`` does (the kernel
used to give such a row loss 0 but still count it and give it a gradient).
The training pods use it (PyTorch's path was eight small kernels per step)."""
from __future__ import annotations

import ctypes

import torch

from vgpu.native import load_kernels

_BOUND = False


def _lib():
    global _BOUND
    lib = load_kernels()
    if not _BOUND:
        vp, ci, cl = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
        lib.vgpu_cross_entropy_fwd_bwd2.argtypes = [vp] * 5 + [cl, ci, cl, cl, cl, cl, cl, ci, vp]
        lib.vgpu_cross_entropy_fwd_bwd2.restype = ci
        lib.vgpu_cross_entropy_rows_workspace.argtypes = [cl, ci]
        lib.vgpu_cross_entropy_rows_workspace.restype = cl
        _BOUND = True
    return lib


def _layout(x: torch.Tensor):
    """(rows, C, hw, bstride, pstride, cstride) of 2-D or 4-D logits, or None."""
    if x.dim() == 2:
        rows, c = x.shape
        if x.stride(1) != 1 or x.stride(0) < c:
            return None
        return rows, c, max(rows, 1), 0, x.stride(0), 1
    if x.dim() == 4:
        b, c, h, w = x.shape
        sb, sc, sh, sw = x.stride()
        if sw * w == sh or h == 1:  # pixels of an image are one linear run
            if x.is_contiguous(memory_format=torch.channels_last) and sc == 1:
                return b * h * w, c, h * w, sb, c, 1
            if x.is_contiguous():
                return b * h * w, c, h * w, sb, 1, sc
    return None


class _CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index, lay):
        rows, c, hw, bs, ps, cs = lay
        lib = _lib()
        loss_rows = torch.empty(lib.vgpu_cross_entropy_rows_workspace(rows, c), dtype=torch.float32,
                                device=logits.device)
        out = torch.empty(2, dtype=torch.float32, device=logits.device)
        dlogits = torch.empty_like(logits)  # same layout as the logits
        p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        rc = lib.vgpu_cross_entropy_fwd_bwd2(p(logits), p(target), p(loss_rows), p(out), p(dlogits), rows, c,
                                                int(ignore_index), hw, bs, ps, cs,
                                                int(logits.dtype == torch.bfloat16),
                                                ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        if rc != 0:
            raise RuntimeError(f"vgpu_cross_entropy_fwd_bwd2: error {rc}")
        ctx.save_for_backward(dlogits, out)
        return out[0]

    @staticmethod
    def backward(ctx, g):
        dlogits, out = ctx.saved_tensors
        # 0-dim scale: the multiply does not promote (one kernel, a bf16 result)
        return dlogits * (g * out[1]), None, None, None


def cross_entropy(logits: torch.Tensor, target: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    """Mean cross-entropy (fp32 scalar) of [rows, C] or [B, C, H, W] logits
    against int64 targets ([rows] or [B, H, W])."""
    lay = None
    if (logits.is_cuda and logits.dtype in (torch.bfloat16, torch.float32) and target.dtype == torch.int64
            and target.is_contiguous() and target.device == logits.device):
        lay = _layout(logits)
        if lay is not None:
            want = (logits.shape[0],) if logits.dim() == 2 else (logits.shape[0], *logits.shape[2:])
            if tuple(target.shape) != want:
                lay = None
    if lay is None:
        return torch.nn.functional.cross_entropy(logits.float(), target, ignore_index=ignore_index)
    return _CrossEntropyFn.apply(logits, target, ignore_index, lay)
