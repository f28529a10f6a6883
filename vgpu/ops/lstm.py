"""Fused LSTM: one input-projection GEMM per layer (hipBLASLt) plus one
persistent recurrence kernel per layer (native/kernels/lstm.hip), instead of
MIOpen's per-timestep kernel sequence.  A 2-layer stack (the ai-benchmark
shape) runs both layers as one wavefront launch -- layer 2 a few steps behind
layer 1, its input projection computed inside the kernel -- in the forward and,
in time-reverse order, in the backward (VGPU_LSTM_WAVE=0: layer by layer).
Inference (`lstm_last_hidden`) and training (`LSTMLayerFn`: forward keeps the activated gates and cells, backward is
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


def _wave(lstm: torch.nn.LSTM) -> bool:
    """Two-layer stacks run as one wavefront launch (lstm2_forward_kernel); VGPU_LSTM_WAVE=0: layer by layer."""
    return lstm.num_layers == 2 and os.environ.get("VGPU_LSTM_WAVE", "1") != "0"


def _flags(b: int, device) -> torch.Tensor:
    return torch.empty(2 * ((b + 15) // 16) + 1, dtype=torch.int32, device=device)


def _p(t):
    return t.data_ptr() if t is not None else None


def lstm_last_hidden(lstm: torch.nn.LSTM, x: torch.Tensor) -> torch.Tensor:
    """h_T of the last layer, [B, H] — what LSTMSentiment reads (y[:, -1])."""
    from vgpu.native import load_kernels
    lib = load_kernels()
    b, t, _ = x.shape
    h = lstm.hidden_size
    stream = torch.cuda.current_stream().cuda_stream
    if _wave(lstm):
        w_ih1, w_hh1 = lstm.weight_ih_l0, lstm.weight_hh_l0.contiguous()
        xp1 = torch.addmm(lstm.bias_ih_l0 + lstm.bias_hh_l0, x.transpose(0, 1).reshape(t * b, -1),
                          w_ih1.t()).view(t, b, 4 * h)
        b2 = (lstm.bias_ih_l1 + lstm.bias_hh_l1).contiguous()
        y1t = torch.empty(t, b, h, dtype=x.dtype, device=x.device)
        xp2 = torch.empty(t, b, 4 * h, dtype=x.dtype, device=x.device)
        hlast = torch.empty(b, h, dtype=x.dtype, device=x.device)
        w_ih2, w_hh2 = lstm.weight_ih_l1.contiguous(), lstm.weight_hh_l1.contiguous()
        flags = _flags(b, x.device)
        rc = lib.vgpu_lstm2_forward(_p(xp1), _p(w_hh1), _p(w_ih2), _p(b2), _p(w_hh2), _p(y1t), _p(xp2), _p(flags),
                                    _p(hlast), None, None, None, None, None, b, t, h, stream)
        _check(rc, "vgpu_lstm2_forward")
        return hlast
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


class LSTM2Fn(torch.autograd.Function):
    """Both layers of a 2-layer stack, batch_first x [B, T, E] -> y2 [B, T, H]
    (zero initial state), forward and backward each one wavefront launch
    (lstm2_forward_kernel / lstm2_backward_kernel) plus the GEMMs around them:
    layer 1's input projection, and the weight / input gradients."""

    @staticmethod
    def forward(ctx, x, w_ih1, w_hh1, b_ih1, b_hh1, w_ih2, w_hh2, b_ih2, b_hh2):
        from vgpu.native import load_kernels
        lib = load_kernels()
        b, t, _ = x.shape
        h = w_hh1.shape[1]
        dev, dt = x.device, x.dtype
        xt = x.transpose(0, 1).reshape(t * b, -1)  # [T*B, E], timestep-major
        xp1 = torch.addmm(b_ih1 + b_hh1, xt, w_ih1.t()).view(t, b, 4 * h)
        w_hh1, w_ih2, w_hh2 = w_hh1.contiguous(), w_ih2.contiguous(), w_hh2.contiguous()
        y1t = torch.empty(t, b, h, dtype=dt, device=dev)
        y2t = torch.empty(t, b, h, dtype=dt, device=dev)
        xp2 = torch.empty(t, b, 4 * h, dtype=dt, device=dev)
        gates1 = torch.empty(t, b, 4 * h, dtype=dt, device=dev)
        gates2 = torch.empty_like(gates1)
        cells1 = torch.empty(t, b, h, dtype=torch.float32, device=dev)
        cells2 = torch.empty_like(cells1)
        # every buffer the kernel touches is held in a local until the launch returns
        # (a temporary freed mid-argument-list can be handed out again to the next one)
        b2 = (b_ih2 + b_hh2).contiguous()
        flags = _flags(b, dev)
        rc = lib.vgpu_lstm2_forward(_p(xp1), _p(w_hh1), _p(w_ih2), _p(b2), _p(w_hh2), _p(y1t), _p(xp2), _p(flags),
                                    None, _p(y2t), _p(gates1), _p(gates2), _p(cells1), _p(cells2), b, t, h,
                                    torch.cuda.current_stream().cuda_stream)
        _check(rc, "vgpu_lstm2_forward")
        ctx.save_for_backward(xt, w_ih1, w_hh1, w_ih2, w_hh2, y1t, y2t, gates1, gates2, cells1, cells2)
        return y2t.transpose(0, 1)

    @staticmethod
    def backward(ctx, dy):
        from vgpu.native import load_kernels
        lib = load_kernels()
        xt, w_ih1, w_hh1, w_ih2, w_hh2, y1t, y2t, gates1, gates2, cells1, cells2 = ctx.saved_tensors
        t, b, h = y1t.shape
        dy = dy.to(y1t.dtype).contiguous()
        dgates1 = torch.empty_like(gates1)
        dgates2 = torch.empty_like(gates2)
        dy1 = torch.empty_like(y1t)
        flags = _flags(b, y1t.device)
        _check(lib.vgpu_lstm2_backward(_p(gates1), _p(cells1), _p(gates2), _p(cells2), _p(dy), _p(w_hh1), _p(w_hh2),
                                       _p(w_ih2), _p(dgates1), _p(dgates2), _p(dy1), _p(flags), b, t, h,
                                       torch.cuda.current_stream().cuda_stream), "vgpu_lstm2_backward")

        def grads(dgates, hs, inp):
            # dW_hh = Σ_t dgates_tᵀ h_{t-1} (h_{-1} = 0), dW_ih = dgatesᵀ · input, db = Σ dgates
            dg = dgates.view(t * b, 4 * h)
            dw_hh = dgates[1:].reshape((t - 1) * b, 4 * h).t() @ hs[:-1].reshape((t - 1) * b, h) if t > 1 \
                else torch.zeros(4 * h, h, dtype=dg.dtype, device=dg.device)
            return dg, dg.t() @ inp, dw_hh, dg.float().sum(0).to(dg.dtype)

        dg2, dw_ih2, dw_hh2, db2 = grads(dgates2, y2t, y1t.view(t * b, h))
        dg1, dw_ih1, dw_hh1, db1 = grads(dgates1, y1t, xt)
        dx = (dg1 @ w_ih1).view(t, b, -1).transpose(0, 1) if ctx.needs_input_grad[0] else None
        return dx, dw_ih1, dw_hh1, db1, db1, dw_ih2, dw_hh2, db2, db2


def lstm_forward_train(lstm: torch.nn.LSTM, x: torch.Tensor) -> torch.Tensor:
    """Output of the last layer [B, T, H], differentiable w.r.t. the LSTM weights."""
    if _wave(lstm):
        return LSTM2Fn.apply(x, lstm.weight_ih_l0, lstm.weight_hh_l0, lstm.bias_ih_l0, lstm.bias_hh_l0,
                             lstm.weight_ih_l1, lstm.weight_hh_l1, lstm.bias_ih_l1, lstm.bias_hh_l1)
    y = x
    for layer in range(lstm.num_layers):
        y = LSTMLayerFn.apply(y, getattr(lstm, f"weight_ih_l{layer}"), getattr(lstm, f"weight_hh_l{layer}"),
                              getattr(lstm, f"bias_ih_l{layer}"), getattr(lstm, f"bias_hh_l{layer}"))
    return y
