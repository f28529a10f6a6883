"""Fused NHWC bf16 epilogues (native/kernels/fused_eltwise.hip) and their
plain-PyTorch fp32 references.

Tensors are NCHW-shaped torch tensors in channels_last memory format (so the
memory order is N,H,W,C and the channel of element i is i % C).
"""
from __future__ import annotations

import ctypes

import torch

from vgpu.native import load_kernels

ACT = {"none": 0, "relu": 1, "relu6": 2}


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _nhwc_ok(t: torch.Tensor) -> None:
    if t.dtype != torch.bfloat16 or not t.is_cuda:
        raise TypeError("expected a bf16 CUDA tensor")
    if t.dim() == 4 and not t.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("expected channels_last memory format")
    if t.dim() == 2 and not t.is_contiguous():
        raise ValueError("expected a contiguous [rows, C] tensor")


def _channels(t: torch.Tensor) -> int:
    return t.shape[1]


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what}: hipError {rc}")


def bias_act_(x: torch.Tensor, bias: torch.Tensor, act: str = "relu") -> torch.Tensor:
    """In place: x = act(x + bias[c]).  bias: fp32 [C]."""
    _nhwc_ok(x)
    assert bias.dtype == torch.float32 and bias.is_contiguous() and bias.numel() == _channels(x)
    _check(load_kernels().vgpu_bias_act_nhwc(x.data_ptr(), bias.data_ptr(), x.numel(), _channels(x),
                                             ACT[act], _stream()), "bias_act")
    return x


def scale_shift_act(x: torch.Tensor, scale: torch.Tensor, shift: torch.Tensor,
                    act: str = "relu", out: torch.Tensor | None = None) -> torch.Tensor:
    _nhwc_ok(x)
    if out is None:
        out = torch.empty_like(x)
    _check(load_kernels().vgpu_scale_shift_act_nhwc(
        x.data_ptr(), out.data_ptr(), scale.data_ptr(), shift.data_ptr(), x.numel(), _channels(x),
        ACT[act], _stream()), "scale_shift_act")
    return out


def add_scale_shift_act(a: torch.Tensor, b: torch.Tensor, scale: torch.Tensor,
                        shift: torch.Tensor, act: str = "relu",
                        out_sum: torch.Tensor | None = None,
                        out_act: torch.Tensor | None = None) -> tuple[torch.Tensor, torch.Tensor]:
    """s = a + b; y = act(s * scale[c] + shift[c]); returns (s, y)."""
    _nhwc_ok(a)
    _nhwc_ok(b)
    assert a.shape == b.shape
    if out_sum is None:
        out_sum = torch.empty_like(a)
    if out_act is None:
        out_act = torch.empty_like(a)
    _check(load_kernels().vgpu_add_scale_shift_act_nhwc(
        a.data_ptr(), b.data_ptr(), out_sum.data_ptr(), out_act.data_ptr(), scale.data_ptr(),
        shift.data_ptr(), a.numel(), _channels(a), ACT[act], _stream()), "add_scale_shift_act")
    return out_sum, out_act


# ---- fp32 references --------------------------------------------------------------
def _act_ref(y: torch.Tensor, act: str) -> torch.Tensor:
    if act == "relu":
        return y.clamp_min(0)
    if act == "relu6":
        return y.clamp(0, 6)
    return y


def _bc(p: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    return p.view(1, -1, *([1] * (x.dim() - 2)))


def bias_act_ref(x, bias, act="relu"):
    return _act_ref(x.float() + _bc(bias.float(), x), act).to(x.dtype)


def scale_shift_act_ref(x, scale, shift, act="relu"):
    return _act_ref(x.float() * _bc(scale.float(), x) + _bc(shift.float(), x), act).to(x.dtype)


def add_scale_shift_act_ref(a, b, scale, shift, act="relu"):
    s = (a.float() + b.float()).to(a.dtype)
    return s, scale_shift_act_ref(s, scale, shift, act)


def bn_scale_shift(bn: torch.nn.BatchNorm2d) -> tuple[torch.Tensor, torch.Tensor]:
    """Eval-mode BatchNorm as per-channel fp32 (scale, shift)."""
    scale = (bn.weight.float() / torch.sqrt(bn.running_var.float() + bn.eps)).contiguous()
    shift = (bn.bias.float() - bn.running_mean.float() * scale).contiguous()
    return scale, shift
