"""Fused LSTM inference: one input-projection GEMM per layer (hipBLASLt) plus
one persistent recurrence kernel per layer (native/kernels/lstm.hip), instead of
MIOpen's per-timestep kernel sequence.  Inference only (the training path keeps
nn.LSTM); hidden size 128 (the ai-benchmark LSTM-Sentiment shape)."""
from __future__ import annotations

import os

import torch


def supported(lstm: torch.nn.LSTM, x: torch.Tensor) -> bool:
    """Inference (no autograd), bf16 on the GPU, the LSTM-Sentiment shape."""
    return (os.environ.get("VGPU_LSTM_FUSED", "1") != "0" and not torch.is_grad_enabled() and x.is_cuda
            and x.dtype == torch.bfloat16 and lstm.hidden_size == 128 and lstm.batch_first
            and not lstm.bidirectional and lstm.proj_size == 0 and lstm.bias)


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
