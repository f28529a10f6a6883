"""Training-mode BatchNorm + activation for NHWC bf16 activations
(native/kernels/bn_nhwc.hip) as an autograd Function, and the module-level
entry `bn_act` the training models call.

    y = act(γ · (x - mean) / sqrt(var + eps) + β),  batch statistics over N·H·W

Forward saves mean / invstd (fp32) and updates the module's running stats
(unbiased variance, PyTorch momentum convention); backward produces dx, dγ, dβ
in one reduction + one elementwise pass, with the activation's derivative
recomputed from x (no saved mask or pre-activation tensor).

Dispatch: a training-mode BatchNorm2d on a 4-D bf16 CUDA channels_last tensor
with C % 8 == 0 runs the native kernels (a missing extension raises
NativeMissing — no silent fallback on a GPU).  Everything else — CPU tensors,
fp32, eval mode, momentum=None — takes the PyTorch path, which is also the
numerics reference (tests/test_gpu_bn.py).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import threading

import torch
import torch.nn.functional as F
from torch import nn

from vgpu.native import load_kernels

ACT = {"none": 0, "relu": 1, "relu6": 2}
_CL = torch.channels_last
# VGPU_NATIVE_BN=0 keeps PyTorch's BatchNorm everywhere (A/B measurements).
_ENABLED = os.environ.get("VGPU_NATIVE_BN", "1") != "0"


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t: torch.Tensor | None):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _param_bf16(*ts: torch.Tensor | None) -> int:
    dts = {t.dtype for t in ts if t is not None}
    if len(dts) > 1:
        raise TypeError(f"BatchNorm parameters of mixed dtypes {dts}")
    dt = dts.pop() if dts else torch.float32
    if dt not in (torch.float32, torch.bfloat16):
        raise TypeError(f"BatchNorm parameters must be fp32 or bf16, got {dt}")
    return int(dt == torch.bfloat16)


def _workspace(lib, m: int, c: int, device) -> torch.Tensor:
    n = lib.vgpu_bn_workspace(m, c)
    if n < 0:
        raise ValueError(f"unsupported BatchNorm shape: rows {m} channels {c}")
    return torch.empty(n, dtype=torch.float32, device=device)


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum: float, eps: float, act: int,
                res_out: bool = False, add: torch.Tensor | None = None):
        lib = load_kernels()
        n, c, h, w = x.shape
        m = n * h * w
        y = torch.empty_like(x, memory_format=_CL)
        mean = torch.empty(c, dtype=torch.float32, device=x.device)
        invstd = torch.empty_like(mean)
        pb = _param_bf16(weight, bias, running_mean, running_var)
        ws = _workspace(lib, m, c, x.device)
        rc = -2
        if add is not None:  # y = act(bn(x)) + add in the same pass when the plan has that form
            rc = lib.vgpu_bn_act_fwd_train_add(
                _ptr(x), _ptr(y), _ptr(weight), _ptr(bias), _ptr(running_mean), _ptr(running_var),
                _ptr(mean), _ptr(invstd), _ptr(ws), m, c, float(eps), float(momentum), act, pb, _ptr(add),
                _stream())
        if rc == -2:
            rc = lib.vgpu_bn_act_fwd_train(
                _ptr(x), _ptr(y), _ptr(weight), _ptr(bias), _ptr(running_mean), _ptr(running_var),
                _ptr(mean), _ptr(invstd), _ptr(ws), m, c, float(eps), float(momentum), act, pb, _stream())
            if rc == 0 and add is not None:
                y.add_(add)
        if rc != 0:
            raise RuntimeError(f"vgpu_bn_act_fwd_train: hipError {rc}")
        ctx.save_for_backward(x, weight, bias, mean, invstd)
        ctx.act = act
        ctx.pb = pb
        ctx.has_add = add is not None
        if res_out:
            # x again, as an output of this node: the gradient it receives (an
            # identity shortcut's) is summed into dx by the backward kernel
            # instead of by a separate autograd add pass over the activation.
            return y, x.view_as(x)
        return y

    @staticmethod
    def backward(ctx, dy, dres=None):
        x, weight, bias, mean, invstd = ctx.saved_tensors
        lib = load_kernels()
        dy = dy.contiguous(memory_format=_CL)
        n, c, h, w = x.shape
        m = n * h * w
        dx = torch.empty_like(x, memory_format=_CL)
        dw = torch.empty_like(weight) if weight is not None and ctx.needs_input_grad[1] else None
        db = torch.empty_like(bias) if bias is not None and ctx.needs_input_grad[2] else None
        if dres is not None:
            dres = dres.contiguous(memory_format=_CL)
        rc = lib.vgpu_bn_act_bwd_add(
            _ptr(dy), _ptr(x), _ptr(dx), _ptr(weight), _ptr(bias), _ptr(mean), _ptr(invstd),
            _ptr(dw), _ptr(db), _ptr(_workspace(lib, m, c, x.device)), m, c, ctx.act, ctx.pb, _ptr(dres),
            _stream())
        if rc != 0:
            raise RuntimeError(f"vgpu_bn_act_bwd: hipError {rc}")
        dadd = dy if ctx.has_add and ctx.needs_input_grad[9] else None  # the shortcut's gradient is dy itself
        return dx, dw, db, None, None, None, None, None, None, dadd


def native_eligible(x: torch.Tensor, bn: nn.BatchNorm2d) -> bool:
    return (_ENABLED and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4
            and x.is_contiguous(memory_format=_CL) and x.shape[1] % 8 == 0
            and x.shape[0] * x.shape[2] * x.shape[3] > 1
            and (bn.training or not bn.track_running_stats)
            and (bn.momentum is not None or not bn.track_running_stats))


def _act(y: torch.Tensor, act: str) -> torch.Tensor:
    if act == "relu":
        return F.relu(y)
    if act == "relu6":
        return F.relu6(y)
    return y


_counters = threading.local()


@contextlib.contextmanager
def batched_step_counters():
    """Defer every native BN's `num_batches_tracked += 1` inside the block to one
    multi-tensor add at exit: one kernel per forward instead of one per layer
    (a ResNet-V2-50 training step launched 41 of them, 190 µs of a 7.8 ms step).
    Same counter values as the module's own update; nests (the outermost block
    flushes)."""
    outer = getattr(_counters, "pending", None)
    if outer is None:
        _counters.pending = []
    try:
        yield
    finally:
        if outer is None:
            pend, _counters.pending = _counters.pending, None
            if pend:
                torch._foreach_add_(pend, 1)


def bn_act(x: torch.Tensor, bn: nn.BatchNorm2d, act: str = "relu",
           add: torch.Tensor | None = None) -> torch.Tensor:
    """act(bn(x)) (+ add) with the module's own semantics (training statistics
    and running-stat update in train mode, running stats in eval mode).  add:
    an identity shortcut summed in the BN's own pass where the kernel plan
    allows (one launch fewer per residual block)."""
    if act not in ACT:
        raise ValueError(act)
    if not native_eligible(x, bn) or (add is not None and (add.shape != x.shape or add.dtype != x.dtype
                                                           or not add.is_contiguous(memory_format=_CL))):
        y = _act(bn(x), act)
        return y if add is None else y + add
    track = bn.track_running_stats and bn.running_mean is not None
    if track:
        pend = getattr(_counters, "pending", None)
        if pend is not None:
            pend.append(bn.num_batches_tracked)
        else:
            bn.num_batches_tracked.add_(1)
    return _BNActFn.apply(x, bn.weight, bn.bias, bn.running_mean if track else None,
                          bn.running_var if track else None, bn.momentum if track else 0.0,
                          bn.eps, ACT[act], False, add)


def bn_act_res(x: torch.Tensor, bn: nn.BatchNorm2d, act: str = "relu") -> tuple[torch.Tensor, torch.Tensor]:
    """(act(bn(x)), x) for a pre-activation block whose identity shortcut is x
    itself: use the returned x as the shortcut, and its gradient is added into
    the BN backward's dx in the same kernel (no separate add over x).  Same
    values as (bn_act(x, bn, act), x)."""
    if act not in ACT:
        raise ValueError(act)
    if not native_eligible(x, bn):
        return _act(bn(x), act), x
    track = bn.track_running_stats and bn.running_mean is not None
    if track:
        pend = getattr(_counters, "pending", None)
        if pend is not None:
            pend.append(bn.num_batches_tracked)
        else:
            bn.num_batches_tracked.add_(1)
    return _BNActFn.apply(x, bn.weight, bn.bias, bn.running_mean if track else None,
                          bn.running_var if track else None, bn.momentum if track else 0.0,
                          bn.eps, ACT[act], True)


def bn_act_reference(x: torch.Tensor, weight, bias, running_mean, running_var, momentum: float,
                     eps: float, act: str) -> torch.Tensor:
    """fp32 PyTorch reference (running stats updated in place, fp32 copies)."""
    y = F.batch_norm(x.float(), running_mean, running_var,
                     None if weight is None else weight.float(), None if bias is None else bias.float(),
                     training=True, momentum=momentum, eps=eps)
    return _act(y, act)
