"""Fused LSTM: one input-projection GEMM per layer (hipBLASLt) plus one
persistent recurrence kernel per layer (native/kernels/lstm.hip), instead of
MIOpen's per-timestep kernel sequence.  Inference (`lstm_last_hidden`) and
training (`LSTMLayerFn`: forward keeps the activated gates and cells, backward is
one backward-through-time kernel plus three GEMMs for the weight and input
gradients).  Hidden size 128 (the ai-benchmark LSTM-Sentiment shape)."""
from __future__ import annotations

import os

import torch


def supported(lstm: torch.nn.LSTM, x: torch.Tensor, training: bool = False) -> bool:
    """bf16 on the GPU, the LSTM-Sentiment shape; inference needs autograd off."""
    return (os.environ.get("VGPU_LSTM_FUSED", "1") != "0" and (training or not torch.is_grad_enabled())
            and x.is_cuda and x.dtype == torch.bfloat16 and lstm.hidden_size == 128 and lstm.batch_first
            and not lstm.bidirectional and lstm.proj_size == 0 and lstm.bias and lstm.dropout == 0)


def lstm_last_hidden(lstm: torch.nn.LSTM, x: torch.Tensor) -> torch.Tensor:
    """h_T of the last layer, [B, H] — what LSTMSentiment reads (y[:, -1])."""
    from vgpu.native import load_kernels
    lib = load_kernels()
    b, t, _ = x.shape
    h = lstm.hidden_size
    stream = torch.cuda.current_stream().cuda_stream
    inp = x
    hlast = torch.empty(b, h, dtype=x.dtype, device=x.device)
    for layer in range(lstm.num_layers):
        w_ih = getattr(lstm, f"weight_ih_l{layer}")
        w_hh = getattr(lstm, f"weight_hh_l{layer}").contiguous()
        bias = getattr(lstm, f"bias_ih_l{layer}") + getattr(lstm, f"bias_hh_l{layer}")
        # [T, B, 4H]: a timestep's rows are contiguous for the recurrence kernel
        xp = torch.addmm(bias, inp.transpose(0, 1).reshape(t * b, -1), w_ih.t()).view(t, b, 4 * h)
        last = layer == lstm.num_layers - 1
        y = None if last else torch.empty(b, t, h, dtype=x.dtype, device=x.device)
        rc = lib.vgpu_lstm_recurrence(xp.data_ptr(), w_hh.data_ptr(), y.data_ptr() if y is not None else None,
                                      hlast.data_ptr() if last else None, b, t, h, stream)
        if rc != 0:
            raise RuntimeError(f"vgpu_lstm_recurrence failed ({rc})")
        inp = y
    return hlast


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc})")


class LSTMLayerFn(torch.autograd.Function):
    """One layer, batch_first x [B, T, E] -> y [B, T, H] (zero initial state)."""

    @staticmethod
    def forward(ctx, x, w_ih, w_hh, b_ih, b_hh):
        from vgpu.native import load_kernels
        lib = load_kernels()
        b, t, _ = x.shape
        h = w_hh.shape[1]
        xt = x.transpose(0, 1).reshape(t * b, -1)  # [T*B, E], timestep-major
        xp = torch.addmm(b_ih + b_hh, xt, w_ih.t()).view(t, b, 4 * h)
        w_hh = w_hh.contiguous()
        y = torch.empty(b, t, h, dtype=x.dtype, device=x.device)
        gates = torch.empty(t, b, 4 * h, dtype=x.dtype, device=x.device)
        cells = torch.empty(t, b, h, dtype=torch.float32, device=x.device)
        _check(lib.vgpu_lstm_forward_train(xp.data_ptr(), w_hh.data_ptr(), y.data_ptr(), gates.data_ptr(),
                                           cells.data_ptr(), b, t, h, torch.cuda.current_stream().cuda_stream),
               "vgpu_lstm_forward_train")
        ctx.save_for_backward(xt, w_ih, w_hh, y, gates, cells)
        return y

    @staticmethod
    def backward(ctx, dy):
        from vgpu.native import load_kernels
        lib = load_kernels()
        xt, w_ih, w_hh, y, gates, cells = ctx.saved_tensors
        b, t, h = y.shape
        dy = dy.contiguous().to(y.dtype)
        dgates = torch.empty(t, b, 4 * h, dtype=y.dtype, device=y.device)
        _check(lib.vgpu_lstm_backward(gates.data_ptr(), cells.data_ptr(), dy.data_ptr(), w_hh.data_ptr(),
                                      dgates.data_ptr(), b, t, h, torch.cuda.current_stream().cuda_stream),
               "vgpu_lstm_backward")
        dg = dgates.view(t * b, 4 * h)
        # h_{t-1} for every step, timestep-major, h_{-1} = 0
        hprev = torch.zeros(t, b, h, dtype=y.dtype, device=y.device)
        hprev[1:] = y.transpose(0, 1)[:-1]
        dw_hh = dg.t() @ hprev.view(t * b, h)
        dw_ih = dg.t() @ xt
        db = dg.float().sum(0).to(y.dtype)
        dx = (dg @ w_ih).view(t, b, -1).transpose(0, 1) if ctx.needs_input_grad[0] else None
        return dx, dw_ih, dw_hh, db, db


def lstm_forward_train(lstm: torch.nn.LSTM, x: torch.Tensor) -> torch.Tensor:
    """Output of the last layer [B, T, H], differentiable w.r.t. the LSTM weights."""
    y = x
    for layer in range(lstm.num_layers):
        y = LSTMLayerFn.apply(y, getattr(lstm, f"weight_ih_l{layer}"), getattr(lstm, f"weight_hh_l{layer}"),
                              getattr(lstm, f"bias_ih_l{layer}"), getattr(lstm, f"bias_hh_l{layer}"))
    return y
