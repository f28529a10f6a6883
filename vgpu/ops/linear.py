"""Fully connected layers at batch ≤ 8 on the native skinny kernels
(native/kernels/skinny.hip): forward with bias + activation, data gradient
and weight / bias gradients, each one pass over the [N, K] weight, with the
activation's derivative taken from the layer's own output.  VGG-16 training
at batch 2 (test 3.2) runs its classifier this way: hipBLASLt spent 75 / 50 /
66 us on fc1's three GEMMs against a 26 us bound each (profiles/r5/train)."""
from __future__ import annotations

import ctypes

import torch
from torch import nn

from vgpu.native import load_kernels

_ACTS = {"none": 0, "relu": 1, "relu6": 2}
_BOUND = False


def _lib():
    global _BOUND
    lib = load_kernels()
    if not _BOUND:
        vp, ci = ctypes.c_void_p, ctypes.c_int
        lib.vgpu_skinny_supported.argtypes = [ci] * 3
        lib.vgpu_skinny_supported.restype = ci
        lib.vgpu_skinny_fwd.argtypes = [vp] * 4 + [ci] * 4 + [vp]
        lib.vgpu_skinny_fwd.restype = ci
        lib.vgpu_skinny_dgrad_workspace.argtypes = [ci] * 3
        lib.vgpu_skinny_dgrad_workspace.restype = ctypes.c_int64
        lib.vgpu_skinny_dgrad.argtypes = [vp] * 5 + [ctypes.c_int64] + [ci] * 4 + [vp]
        lib.vgpu_skinny_dgrad.restype = ci
        lib.vgpu_skinny_wgrad.argtypes = [vp] * 5 + [ci] * 4 + [vp]
        lib.vgpu_skinny_wgrad.restype = ci
        lib.vgpu_skinny_backward.argtypes = [vp] * 8 + [ctypes.c_int64] + [ci] * 4 + [vp]
        lib.vgpu_skinny_backward.restype = ci
        lib.vgpu_skinny_backward_sgd.argtypes = ([vp] * 8 + [ctypes.c_int64] + [ci] * 4 + [ctypes.c_float] * 4
                                                 + [ci] * 2 + [vp])
        lib.vgpu_skinny_backward_sgd.restype = ci
        _BOUND = True
    return lib


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: error {rc}")


class _SkinnyLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act: int):
        bsz, k = x.shape
        n = w.shape[0]
        y = torch.empty((bsz, n), dtype=x.dtype, device=x.device)
        _check(_lib().vgpu_skinny_fwd(_p(x), _p(w), _p(b), _p(y), bsz, n, k, act, _stream()), "vgpu_skinny_fwd")
        ctx.save_for_backward(x, w, y)
        ctx.act, ctx.has_b = act, b is not None
        ctx.sgd = getattr(w, "_vgpu_sgd", None)  # vgpu.ops.optim.SGD.fuse_into_backward
        ctx.param = w if ctx.sgd is not None else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        dy = dy.contiguous()
        bsz, k = x.shape
        n = w.shape[0]
        lib = _lib()
        yo = y if ctx.act else None
        dx = dw = db = None
        if ctx.sgd is not None and ctx.needs_input_grad[0] and ctx.needs_input_grad[1]:
            done = _backward_sgd(ctx, dy, x, yo, bsz, n, k)
            if done is not None:
                return done
        if ctx.needs_input_grad[0] and ctx.needs_input_grad[1]:  # both: two launches in all
            need = lib.vgpu_skinny_dgrad_workspace(bsz, n, k)
            ws = torch.empty(need // 4, dtype=torch.float32, device=x.device)
            dx, dw = torch.empty_like(x), torch.empty_like(w)
            db = torch.empty(n, dtype=w.dtype, device=w.device) if ctx.has_b else None
            _check(lib.vgpu_skinny_backward(_p(dy), _p(yo), _p(x), _p(w), _p(dx), _p(dw), _p(db), _p(ws), need, bsz,
                                            n, k, ctx.act, _stream()), "vgpu_skinny_backward")
            return dx, dw, db, None
        if ctx.needs_input_grad[0]:
            need = lib.vgpu_skinny_dgrad_workspace(bsz, n, k)
            ws = torch.empty(need // 4, dtype=torch.float32, device=x.device)
            dx = torch.empty_like(x)
            _check(lib.vgpu_skinny_dgrad(_p(dy), _p(yo), _p(w), _p(dx), _p(ws), need, bsz, n, k, ctx.act,
                                         _stream()), "vgpu_skinny_dgrad")
        if ctx.needs_input_grad[1] or (ctx.has_b and ctx.needs_input_grad[2]):
            dw = torch.empty_like(w)
            db = torch.empty(n, dtype=w.dtype, device=w.device) if ctx.has_b else None
            _check(lib.vgpu_skinny_wgrad(_p(dy), _p(yo), _p(x), _p(dw), _p(db), bsz, n, k, ctx.act, _stream()),
                   "vgpu_skinny_wgrad")
        return dx, dw, db, None


def _backward_sgd(ctx, dy, x, yo, bsz, n, k):
    """The weight's SGD step inside its backward (no dW in memory): the
    weight and its momentum buffer are updated in place once the data
    gradient has read the weight; the weight's .grad stays None, so the
    optimizer's own step skips it.  None when the group's settings need the
    unfused path."""
    opt, group = ctx.sgd
    p = ctx.param
    if group["momentum"] == 0 or group["maximize"] or p.numel() % 8:
        return None
    state = opt.state[p]
    buf = state.get("momentum_buffer")
    first = buf is None
    if first:
        buf = torch.empty_like(p)
    if buf.stride() != p.stride() or buf.dtype != p.dtype:
        return None
    lib = _lib()
    need = lib.vgpu_skinny_dgrad_workspace(bsz, n, k)
    ws = torch.empty(need // 4, dtype=torch.float32, device=x.device)
    dx = torch.empty_like(x)
    db = torch.empty(n, dtype=p.dtype, device=p.device) if ctx.has_b else None
    _check(lib.vgpu_skinny_backward_sgd(_p(dy), _p(yo), _p(x), _p(p), _p(dx), _p(buf), _p(db), _p(ws), need, bsz, n,
                                        k, ctx.act, group["lr"], group["momentum"], group["dampening"],
                                        group["weight_decay"], int(group["nesterov"]), int(first), _stream()),
           "vgpu_skinny_backward_sgd")
    if first:
        state["momentum_buffer"] = buf
    p.grad = None
    return dx, None, db, None


def eligible(x: torch.Tensor, lin: nn.Linear) -> bool:
    w = lin.weight
    return (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dim() == 2
            and x.is_contiguous() and w.is_contiguous()
            and (lin.bias is None or (lin.bias.dtype == torch.bfloat16 and lin.bias.is_contiguous()))
            and bool(_lib().vgpu_skinny_supported(x.shape[0], w.shape[0], w.shape[1])))


def linear_act(x: torch.Tensor, lin: nn.Linear, act: str = "none") -> torch.Tensor:
    """act(lin(x)) on the skinny kernels when eligible (batch 1-4 or 8, bf16,
    K % 8 == 0, N even), else through the module."""
    if not eligible(x, lin):
        y = lin(x)
        return torch.relu(y) if act == "relu" else (torch.clamp(y, 0, 6) if act == "relu6" else y)
    return _SkinnyLinearFn.apply(x, lin.weight, lin.bias, _ACTS[act])
