"""Training BatchNorm whose statistics ride on the convolutions around it
(native/kernels/conv_gemm.hip vgpu_conv2d_nhwc_bn, native/kernels/bn_nhwc.hip
vgpu_bn_*_partials).

A pre-activation ResNet block is conv → BN → act → conv → BN → act → conv.
The plain training path (vgpu.ops.bn) reads every BN input once more per
direction just to reduce it: forward Σx / Σx² before the apply pass, backward
Σdz / Σdz·x̂ over x and dy before the dx pass — 29 % of a ResNet-V2-50 step
was BatchNorm, the backward reduction alone 8.7 %
(profiles/r4/train/rocprof_train_1.2_steady_r4.txt).  Here:

* forward: the conv that produces a BN's input also writes (Σz, Σz²) per
  64-row group from its epilogue, and the BN runs finalize + apply only;
* backward: the data gradient of the conv that consumes a BN's output loads x
  in its epilogue, stores dz = dy·act'(x·s + t) instead of dy and writes
  (Σdz, Σdz·x̂) per group; the BN runs finalize + one dx pass.

One autograd node per BN + following conv (`bn_conv`), plus `conv_stats` for a
conv whose input has no BN of its own (a projection block's conv1).  Shapes
the fused kernels do not take (stride-2 data gradients go to MIOpen, the
prologue / narrow kernels) run the unfused pieces inside the same node.

Numerics: partial sums are fp32 over 64 rows, merged in fp64 (unshifted: the
forward uses E[z²] - E[z]², fine for conv outputs whose |mean| is within a few
std); the values summed are the stored bf16 ones, as the unfused path sees them.
tests/test_gpu_bn.py compares both directions with the fp32 PyTorch reference.

On by default in vgpu.models.resnet training (1.2: 2 760 -> 2 991 images/s, 2.2:
815 -> 909, profiles/r4/train/bnfuse/); VGPU_BN_FUSE=0 runs the unfused path (A/B).
"""
from __future__ import annotations

import os

import torch
from torch import nn

from vgpu.native import load_kernels
from vgpu.ops import bn as B
from vgpu.ops.conv import _dgrad_filter, conv2d, conv_backward, out_hw, train_eligible

_CL = torch.channels_last
_ENABLED = os.environ.get("VGPU_BN_FUSE", "1") != "0"
# 3x3 data gradients with the BN statistics take the per-tap LDS-DMA kernel, not
# the (faster) halo-tile kernel; VGPU_BN_FUSE_3X3=0 keeps those on halo + the
# unfused BN backward instead (A/B).
_FUSE_3X3 = os.environ.get("VGPU_BN_FUSE_3X3", "1") != "0"


def enabled() -> bool:
    return _ENABLED


def set_enabled(on: bool) -> None:
    global _ENABLED
    _ENABLED = bool(on)


def _groups(m: int) -> int:
    return (m + 63) // 64


def _conv_out(x: torch.Tensor, w: torch.Tensor, stride: int, padding: int, residual, want_stats: bool):
    """z = conv(x, w) (+ residual), and its (Σz, Σz²) pairs [G, Cout, 2] when the
    LDS-DMA kernels take the shape (else None)."""
    n, c, h, wd = x.shape
    cout, _, ks, _ = w.shape
    oh, ow = out_hw(h, wd, ks, stride, padding)
    z = torch.empty((n, cout, oh, ow), dtype=x.dtype, device=x.device, memory_format=_CL)
    if want_stats:
        st = torch.empty((_groups(n * oh * ow), cout, 2), dtype=torch.float32, device=x.device)
        rc = load_kernels().vgpu_conv2d_nhwc_bn(
            B._ptr(x), B._ptr(w), B._ptr(z), B._ptr(residual), n, h, wd, c, cout, ks, stride, padding,
            B._ptr(st), None, None, 0, 1, B._stream())
        if rc == 0:
            return z, st
        if rc != -1:
            raise RuntimeError(f"vgpu_conv2d_nhwc_bn: error {rc}")
    conv2d(x, w, stride=stride, padding=padding, residual=residual, out=z)
    return z, None


def _none_stats(x: torch.Tensor) -> torch.Tensor:
    return torch.empty(0, dtype=torch.float32, device=x.device)


class _ConvStatsFn(torch.autograd.Function):
    """z = conv(x, w) (+ residual) plus the (Σz, Σz²) pairs of z (empty when the
    kernel could not produce them).  Backward as vgpu.ops.conv._ConvTrainFn."""

    @staticmethod
    def forward(ctx, x, w, residual, stride: int, padding: int):
        z, st = _conv_out(x, w, stride, padding, residual, True)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the statistics output
        ctx.save_for_backward(x, w)
        ctx.stride, ctx.padding, ctx.has_res = stride, padding, residual is not None
        st = st if st is not None else _none_stats(x)
        ctx.mark_non_differentiable(st)
        return z, st

    @staticmethod
    def backward(ctx, dz, _dst):
        x, w = ctx.saved_tensors
        if dz is None:
            return None, None, None, None, None
        dz = dz.contiguous(memory_format=_CL)
        dx, dw = conv_backward(dz, x, w, ctx.stride, ctx.padding, ctx.needs_input_grad[0], ctx.needs_input_grad[1])
        dres = dz if ctx.has_res and ctx.needs_input_grad[2] else None
        return dx, dw, dres, None, None


class _BNConvFn(torch.autograd.Function):
    """z = conv(act(bn(x)), w) (+ residual), with
    stats_in: (Σx, Σx²) pairs of x from its producer's epilogue (empty: reduce here),
    stats_out: also return z's pairs for the next BN,
    extra output (third): with res_out, x itself, whose gradient (an identity
    shortcut's) is summed into dx by the BN's dx pass; with a shortcut weight
    wsc, the projection shortcut conv(act(bn(x)), wsc, stride sc_stride), whose
    data gradient is added to conv's in the fused epilogue."""

    @staticmethod
    def forward(ctx, x, gamma, beta, run_mean, run_var, w, residual, stats_in, wsc, momentum: float, eps: float,
                act: int, stride: int, padding: int, sc_stride: int, stats_out: bool, res_out: bool):
        lib = load_kernels()
        n, c, h, wd = x.shape
        m = n * h * wd
        pb = B._param_bf16(gamma, beta, run_mean, run_var)
        y = torch.empty_like(x, memory_format=_CL)
        coef = torch.empty(4 * c, dtype=torch.float32, device=x.device)  # s, t, mean, invstd
        if stats_in.numel():
            if tuple(stats_in.shape) != (_groups(m), c, 2):
                raise ValueError(f"stats_in {tuple(stats_in.shape)} for x {tuple(x.shape)}")
            rc = lib.vgpu_bn_act_fwd_partials(
                B._ptr(stats_in), stats_in.shape[0], B._ptr(x), B._ptr(y), B._ptr(gamma), B._ptr(beta),
                B._ptr(run_mean), B._ptr(run_var), B._ptr(coef), m, c, float(eps), float(momentum), act, pb,
                B._stream())
            if rc != 0:
                raise RuntimeError(f"vgpu_bn_act_fwd_partials: hipError {rc}")
        else:
            rc = lib.vgpu_bn_act_fwd_train_coef(
                B._ptr(x), B._ptr(y), B._ptr(gamma), B._ptr(beta), B._ptr(run_mean), B._ptr(run_var),
                B._ptr(coef), B._ptr(B._workspace(lib, m, c, x.device)), m, c, float(eps), float(momentum), act,
                pb, B._stream())
            if rc != 0:
                raise RuntimeError(f"vgpu_bn_act_fwd_train_coef: hipError {rc}")
        z, st = _conv_out(y, w, stride, padding, residual, stats_out)
        # Undefined output gradients stay None: autograd would otherwise zero-fill
        # one fp32 tensor per node for the statistics output (50 fills, 3.5 % of
        # a ResNet-V2-50 step, profiles/r4/train/rocprof_train_1.2_fused_r4.md).
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(x, y, w, gamma, beta, coef, wsc)
        ctx.act, ctx.pb, ctx.stride, ctx.padding, ctx.sc_stride = act, pb, stride, padding, sc_stride
        ctx.has_res = residual is not None
        st = st if st is not None else _none_stats(x)
        ctx.mark_non_differentiable(st)
        if res_out:
            return z, st, x.view_as(x)
        if wsc is not None:
            return z, st, conv2d(y, wsc, stride=sc_stride, padding=0)
        return z, st

    @staticmethod
    def backward(ctx, dz, _dst, dextra=None):
        x, y, w, gamma, beta, coef, wsc = ctx.saved_tensors
        lib = load_kernels()
        if dz is None:  # only the extra output was used
            n_, _, h_, w_ = x.shape
            oh, ow = out_hw(h_, w_, w.shape[2], ctx.stride, ctx.padding)
            dz = torch.zeros((n_, w.shape[0], oh, ow), dtype=x.dtype, device=x.device, memory_format=_CL)
        dz = dz.contiguous(memory_format=_CL)
        n, c, h, wd = x.shape
        m = n * h * wd
        s, p = ctx.stride, ctx.padding
        cout, _, ks, _ = w.shape
        dxres = dysc = dwsc = None
        res_stride = 1
        if dextra is not None:
            dextra = dextra.contiguous(memory_format=_CL)
            if wsc is None:
                dxres = dextra
            elif ctx.sc_stride == 2 and wsc.shape[2] == 1 and s == 1:
                # 1x1 / stride-2 shortcut: its data gradient is a 1x1 GEMM on the
                # compact grid, added at the even pixels by the fused epilogue
                # (no MIOpen transposed conv, no 3/4-zero full-size tensor)
                dysc = conv2d(dextra, _dgrad_filter(wsc))
                res_stride = 2
                _, dwsc = conv_backward(dextra, y, wsc, 2, 0, False, ctx.needs_input_grad[8])
            else:
                # the shortcut's own gradients: dw now, its data gradient joins conv's below
                dysc, dwsc = conv_backward(dextra, y, wsc, ctx.sc_stride, 0, True, ctx.needs_input_grad[8])
                dysc = dysc.contiguous(memory_format=_CL)
        need_dx = any(ctx.needs_input_grad[:3])
        dgamma = torch.empty_like(gamma) if gamma is not None and ctx.needs_input_grad[1] else None
        dbeta = torch.empty_like(beta) if beta is not None and ctx.needs_input_grad[2] else None
        mean, invstd = coef[2 * c:3 * c], coef[3 * c:]
        dx = torch.empty_like(x, memory_format=_CL) if need_dx else None
        fused = False
        if need_dx and s == 1 and (ks == 1 or _FUSE_3X3):
            # data gradient of the conv (+ the shortcut's) with the BN backward's reduction in its epilogue
            dpre = torch.empty_like(x, memory_format=_CL)
            part = torch.empty((_groups(m), c, 2), dtype=torch.float32, device=x.device)
            oh, ow = dz.shape[2], dz.shape[3]
            rc = lib.vgpu_conv2d_nhwc_bn(
                B._ptr(dz), B._ptr(_dgrad_filter(w)), B._ptr(dpre), B._ptr(dysc), n, oh, ow, cout, c, ks, 1,
                ks - 1 - p, B._ptr(part), B._ptr(x), B._ptr(coef), ctx.act, res_stride, B._stream())
            if rc == 0:
                ws = torch.empty(4 * c, dtype=torch.float32, device=x.device)
                rc = lib.vgpu_bn_bwd_partials(
                    B._ptr(part), part.shape[0], B._ptr(dpre), B._ptr(x), B._ptr(dx), B._ptr(gamma), B._ptr(beta),
                    B._ptr(mean), B._ptr(invstd), B._ptr(dgamma), B._ptr(dbeta), B._ptr(ws), m, c, ctx.pb,
                    B._ptr(dxres), B._stream())
                if rc != 0:
                    raise RuntimeError(f"vgpu_bn_bwd_partials: hipError {rc}")
                fused = True
            elif rc != -1:
                raise RuntimeError(f"vgpu_conv2d_nhwc_bn (backward): error {rc}")
        dy_bn, dw = conv_backward(dz, y, w, s, p, need_dx and not fused, ctx.needs_input_grad[5])
        if need_dx and not fused:
            dy_bn = dy_bn.contiguous(memory_format=_CL)
            if dysc is not None and res_stride == 2:
                dy_bn = dy_bn.clone()
                dy_bn[:, :, ::2, ::2] += dysc
            elif dysc is not None:
                dy_bn = dy_bn + dysc
            rc = lib.vgpu_bn_act_bwd_add(
                B._ptr(dy_bn), B._ptr(x), B._ptr(dx), B._ptr(gamma), B._ptr(beta), B._ptr(mean), B._ptr(invstd),
                B._ptr(dgamma), B._ptr(dbeta), B._ptr(B._workspace(lib, m, c, x.device)), m, c, ctx.act, ctx.pb,
                B._ptr(dxres), B._stream())
            if rc != 0:
                raise RuntimeError(f"vgpu_bn_act_bwd: hipError {rc}")
        dres = dz if ctx.has_res and ctx.needs_input_grad[6] else None
        return (dx, dgamma, dbeta, None, None, dw, dres, None, dwsc, None, None, None, None, None, None, None, None)


def eligible(x: torch.Tensor, bn: nn.BatchNorm2d | None, conv: nn.Conv2d) -> bool:
    return (_ENABLED and train_eligible(x, conv) and conv.in_channels % 64 == 0
            and (bn is None or (B.native_eligible(x, bn) and bn.training)))


def _bump(bn: nn.BatchNorm2d) -> bool:
    track = bn.track_running_stats and bn.running_mean is not None
    if track:
        pend = getattr(B._counters, "pending", None)
        if pend is not None:
            pend.append(bn.num_batches_tracked)
        else:
            bn.num_batches_tracked.add_(1)
    return track


def bn_conv(x: torch.Tensor, bn: nn.BatchNorm2d, conv: nn.Conv2d, *, act: str = "relu",
            residual: torch.Tensor | None = None, stats_in: torch.Tensor | None = None,
            stats_out: bool = True, res_out: bool = False, shortcut: nn.Conv2d | None = None):
    """(conv(act(bn(x))) + residual, its statistics or None[, x | shortcut(act(bn(x)))])
    — see the module docstring.  Call only when eligible(x, bn, conv) (and, with
    a shortcut, eligible(x, None, shortcut): 1x1, no padding)."""
    if res_out and shortcut is not None:
        raise ValueError("res_out and shortcut are exclusive")
    track = _bump(bn)
    outs = _BNConvFn.apply(
        x, bn.weight, bn.bias, bn.running_mean if track else None, bn.running_var if track else None,
        conv.weight, residual, stats_in if stats_in is not None else _none_stats(x),
        shortcut.weight if shortcut is not None else None,
        bn.momentum if track else 0.0, bn.eps, B.ACT[act], conv.stride[0], conv.padding[0],
        shortcut.stride[0] if shortcut is not None else 1, stats_out, res_out)
    st = outs[1] if outs[1].numel() else None
    return (outs[0], st, outs[2]) if len(outs) == 3 else (outs[0], st)


def conv_stats(x: torch.Tensor, conv: nn.Conv2d, residual: torch.Tensor | None = None):
    """(conv(x) + residual, its statistics or None).  Call only when eligible(x, None, conv)."""
    z, st = _ConvStatsFn.apply(x, conv.weight, residual, conv.stride[0], conv.padding[0])
    return z, (st if st.numel() else None)
