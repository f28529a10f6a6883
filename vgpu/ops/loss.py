"""Mean cross-entropy over logits with integer targets on one native kernel
pass (native/kernels/loss.hip): the forward also writes dlogits, so the
backward is a single scale by the incoming gradient.  Same value and
gradient as torch.nn.functional.cross_entropy(logits.float(), target)
(reduction 'mean', no weights / ignore_index / label smoothing); the
training pods use it (PyTorch's path was eight small kernels per step)."""
from __future__ import annotations

import ctypes

import torch

from vgpu.native import load_kernels

_BOUND = False


def _lib():
    global _BOUND
    lib = load_kernels()
    if not _BOUND:
        vp, ci = ctypes.c_void_p, ctypes.c_int
        lib.vgpu_cross_entropy_fwd_bwd.argtypes = [vp] * 5 + [ci] * 3 + [vp]
        lib.vgpu_cross_entropy_fwd_bwd.restype = ci
        _BOUND = True
    return lib


class _CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target):
        rows, c = logits.shape
        loss_rows = torch.empty(rows, dtype=torch.float32, device=logits.device)
        loss = torch.empty((), dtype=torch.float32, device=logits.device)
        dlogits = torch.empty_like(logits)
        p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        rc = _lib().vgpu_cross_entropy_fwd_bwd(p(logits), p(target), p(loss_rows), p(loss), p(dlogits), rows, c,
                                               int(logits.dtype == torch.bfloat16),
                                               ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        if rc != 0:
            raise RuntimeError(f"vgpu_cross_entropy_fwd_bwd: error {rc}")
        ctx.save_for_backward(dlogits)
        return loss

    @staticmethod
    def backward(ctx, g):
        (dlogits,) = ctx.saved_tensors
        # g is 0-dim: it scales without promoting, one kernel and a bf16 result
        return dlogits * g, None


def cross_entropy(logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """Mean cross-entropy (fp32 scalar) of [rows, C] logits against int64 targets."""
    if (logits.is_cuda and logits.dim() == 2 and logits.dtype in (torch.bfloat16, torch.float32)
            and logits.is_contiguous() and target.dtype == torch.int64 and target.dim() == 1
            and target.is_contiguous() and target.shape[0] == logits.shape[0]):
        return _CrossEntropyFn.apply(logits, target)
    return torch.nn.functional.cross_entropy(logits.float(), target)
