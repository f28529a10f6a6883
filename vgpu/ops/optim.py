"""SGD with momentum on the native one-launch kernel (native/kernels/optim.hip).

Same update as torch.optim.SGD (momentum, dampening, weight decay, Nesterov;
the momentum buffer starts as the first gradient), for bf16 CUDA parameters
with a dense gradient: every ≤ 48 such tensors of a group are updated by one
kernel whose segment table travels in the kernel arguments (hipGraph-safe).
Anything else (other dtypes, sparse or odd-sized tensors, momentum 0,
maximize) takes PyTorch's own functional SGD.  The training pods use it:
PyTorch's fused SGD moved VGG-16's parameters at ~3.9 TB/s in 7 launches,
15 % of the batch-2 step (profiles/r5/train).
"""
from __future__ import annotations

import ctypes

import torch
from torch.optim.sgd import sgd as _torch_sgd

from vgpu.native import load_kernels

_BOUND = False


def _lib():
    global _BOUND
    lib = load_kernels()
    if not _BOUND:
        vp = ctypes.c_void_p
        lib.vgpu_sgd_bf16.argtypes = [vp, vp, vp, vp, ctypes.c_int] + [ctypes.c_float] * 4 + [ctypes.c_int] * 2 + [vp]
        lib.vgpu_sgd_bf16.restype = ctypes.c_int
        lib.vgpu_sgd_max_segments.restype = ctypes.c_int
        _BOUND = True
    return lib


def _dense(t: torch.Tensor) -> bool:
    return t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last))


def _native_ok(p: torch.Tensor, buf: torch.Tensor | None) -> bool:
    """The update is elementwise over storage: p, its gradient and its momentum
    buffer must be dense with identical strides (channels_last conv weights
    included), bf16, 16-B aligned, numel % 8 == 0."""
    g = p.grad
    return (p.is_cuda and p.dtype == torch.bfloat16 and g is not None and not g.is_sparse
            and g.dtype == torch.bfloat16 and _dense(p) and g.stride() == p.stride()
            and (buf is None or buf.stride() == p.stride())
            and p.numel() % 8 == 0 and p.data_ptr() % 16 == 0 and g.data_ptr() % 16 == 0)


def sgd_bf16_(params: list[torch.Tensor], grads: list[torch.Tensor], bufs: list[torch.Tensor], *, lr: float,
              momentum: float, dampening: float, weight_decay: float, nesterov: bool, first: bool) -> None:
    """In-place native SGD step over bf16 tensors (bufs: momentum buffers,
    written from the gradient when first)."""
    lib = _lib()
    cap = lib.vgpu_sgd_max_segments()
    stream = ctypes.c_void_p(torch.cuda.current_stream(params[0].device).cuda_stream)
    for s in range(0, len(params), cap):
        ps, gs, ms = params[s:s + cap], grads[s:s + cap], bufs[s:s + cap]
        k = len(ps)
        arr = ctypes.c_void_p * k
        rc = lib.vgpu_sgd_bf16(arr(*[t.data_ptr() for t in ps]), arr(*[t.data_ptr() for t in gs]),
                               arr(*[t.data_ptr() for t in ms]), (ctypes.c_int64 * k)(*[t.numel() for t in ps]),
                               k, lr, momentum, dampening, weight_decay, int(nesterov), int(first), stream)
        if rc != 0:
            raise RuntimeError(f"vgpu_sgd_bf16: error {rc}")


class SGD(torch.optim.Optimizer):
    """torch.optim.SGD with bf16 parameters updated by the native kernel."""

    def __init__(self, params, lr: float = 1e-3, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False, maximize: bool = False):
        if lr < 0 or momentum < 0 or weight_decay < 0:
            raise ValueError("lr, momentum and weight_decay must be >= 0")
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening,
                                      weight_decay=weight_decay, nesterov=nesterov, maximize=maximize))

    def fuse_into_backward(self, module: torch.nn.Module) -> int:
        """Optimizer-in-backward for the module's fully connected weights: a
        registered weight that goes through the skinny kernels
        (vgpu.ops.linear, batch ≤ 8) is updated inside its own backward and its
        gradient never reaches memory (VGG-16 at batch 2: 2 x 247 MB of dW
        traffic less per step).  Only for weights used once per step and no
        gradient accumulation across backward passes.  A registered weight that
        takes any other path keeps an ordinary gradient and is stepped here.
        Not under data parallelism: the gradient that a collective would
        average never exists (refused when a process group of more than one
        rank is up).  Returns the number of weights registered."""
        if torch.distributed.is_available() and torch.distributed.is_initialized() \
                and torch.distributed.get_world_size() > 1:
            raise ValueError("fuse_into_backward: the gradients of a data-parallel step must reach the collectives")
        count = 0
        for group in self.param_groups:
            ids = {id(p) for p in group["params"]}
            for m in module.modules():
                if isinstance(m, torch.nn.Linear) and id(m.weight) in ids:
                    m.weight._vgpu_sgd = (self, group)
                    count += 1
        return count

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            hp = dict(lr=group["lr"], momentum=group["momentum"], dampening=group["dampening"],
                      weight_decay=group["weight_decay"], nesterov=group["nesterov"])
            native = group["momentum"] != 0 and not group["maximize"]
            first_p, cont_p, rest = [], [], []
            for p in group["params"]:
                if p.grad is None:
                    continue
                buf = self.state[p].get("momentum_buffer")
                if native and _native_ok(p, buf):
                    (first_p if buf is None else cont_p).append(p)
                else:
                    rest.append(p)
            for ps, first in ((first_p, True), (cont_p, False)):
                if not ps:
                    continue
                if first:
                    for p in ps:
                        self.state[p]["momentum_buffer"] = torch.empty_like(p, memory_format=torch.preserve_format)
                bufs = [self.state[p]["momentum_buffer"] for p in ps]
                sgd_bf16_(ps, [p.grad for p in ps], bufs, first=first, **hp)
            if rest:
                bufs = [self.state[p].get("momentum_buffer") for p in rest]
                _torch_sgd(rest, [p.grad for p in rest], bufs, weight_decay=group["weight_decay"],
                           momentum=group["momentum"], lr=group["lr"], dampening=group["dampening"],
                           nesterov=group["nesterov"], maximize=group["maximize"])
                if group["momentum"] != 0:
                    for p, b in zip(rest, bufs):
                        self.state[p]["momentum_buffer"] = b
        return loss
