"""MFMA implicit-GEMM NHWC convolution with fused prologue / epilogue
(native/kernels/conv_gemm.hip) and its fp32 PyTorch reference.

    y = act(conv(pro(x), w) + bias + residual),   pro(x) = relu(x * scale[c] + shift[c])

Tensors: bf16, NCHW-shaped, channels_last memory.  Supported: 1x1 and 3x3
filters, any stride / padding, C % 64 == 0 and Cout % 64 == 0 (every
convolution of ResNet-V2 after the stem), plus the narrow 4x4 C=16 form the
stem takes after space-to-depth (stem_conv).  No silent fallback: unsupported
shapes raise, a missing extension raises NativeMissing.
"""
from __future__ import annotations

import ctypes
import os
import weakref

import torch
import torch.nn.functional as F

from vgpu.native import load_kernels

_CL = torch.channels_last


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t: torch.Tensor | None):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _nhwc(t: torch.Tensor, name: str) -> None:
    if t.dtype != torch.bfloat16 or not t.is_cuda or t.dim() != 4:
        raise TypeError(f"{name}: expected a 4-D bf16 CUDA tensor")
    if not t.is_contiguous(memory_format=_CL):
        raise ValueError(f"{name}: expected channels_last memory format")


def supported(c: int, cout: int, ks: int) -> bool:
    return cout % 64 == 0 and ((c % 64 == 0 and ks in (1, 3)) or (c == 16 and ks == 4))


def out_hw(h: int, w: int, ks: int, stride: int, pad: int) -> tuple[int, int]:
    return (h + 2 * pad - ks) // stride + 1, (w + 2 * pad - ks) // stride + 1


_ACTS = {"none": 0, "relu": 1, "relu6": 2}  # the kernels' epilogue activation codes


def conv2d(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None, *,
           stride: int = 1, padding: int = 0, act: str = "none",
           pro: tuple[torch.Tensor, torch.Tensor] | None = None,
           residual: torch.Tensor | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """x [N,C,H,W] bf16 channels_last; w [Cout,C,k,k] bf16 channels_last;
    bias fp32 or bf16 [Cout]; pro = (scale, shift) fp32 [C] (BN+ReLU on the input);
    residual [N,Cout,OH,OW] bf16 channels_last; act 'none' | 'relu' | 'relu6'.
    Convs whose output tiles cannot fill the GPU run split-K (a workspace from
    the caching allocator, vgpu_conv2d_workspace)."""
    _nhwc(x, "x")
    _nhwc(w, "w")
    n, c, h, wd = x.shape
    cout, cw, ks, ks2 = w.shape
    if cw != c or ks != ks2 or not supported(c, cout, ks):
        raise ValueError(f"unsupported conv: x {tuple(x.shape)} w {tuple(w.shape)}")
    oh, ow = out_hw(h, wd, ks, stride, padding)
    if act not in _ACTS:
        raise ValueError(act)
    for p in (pro if pro is not None else ()):
        if p.dtype != torch.float32 or not p.is_contiguous() or not p.is_cuda:
            raise TypeError("prologue parameters must be contiguous fp32 CUDA tensors")
    if bias is not None and (bias.dtype not in (torch.float32, torch.bfloat16) or not bias.is_contiguous()
                             or not bias.is_cuda):
        raise TypeError("bias must be a contiguous fp32 or bf16 CUDA tensor")
    if bias is not None and bias.numel() != cout:
        raise ValueError("bias size")
    if pro is not None and (pro[0].numel() != c or pro[1].numel() != c):
        raise ValueError("prologue size")
    if residual is not None:
        _nhwc(residual, "residual")
        if tuple(residual.shape) != (n, cout, oh, ow):
            raise ValueError("residual shape")
    if out is None:
        out = torch.empty((n, cout, oh, ow), dtype=x.dtype, device=x.device, memory_format=_CL)
    else:
        _nhwc(out, "out")
    lib = load_kernels()
    key = (n, h, wd, c, cout, ks, stride, padding, pro is not None)
    need = _WS_BYTES.get(key)
    if need is None:
        need = _WS_BYTES[key] = lib.vgpu_conv2d_workspace(*key[:-1], int(pro is not None))
    ws = torch.empty(need // 4, dtype=torch.float32, device=x.device) if need > 0 else None
    code = _ACTS[act] | (256 if bias is not None and bias.dtype == torch.bfloat16 else 0)
    rc = lib.vgpu_conv2d_nhwc_ws(
        _ptr(x), _ptr(w), _ptr(out), _ptr(residual), _ptr(bias),
        _ptr(pro[0] if pro else None), _ptr(pro[1] if pro else None),
        n, h, wd, c, cout, ks, stride, padding, code, _ptr(ws), need, _stream())
    if rc != 0:
        raise RuntimeError(f"vgpu_conv2d_nhwc: error {rc}")
    return out


_WS_BYTES: dict[tuple, int] = {}  # conv shape -> split-K workspace bytes (0: unsplit)


def set_splitk(mode: int) -> None:
    """A/B switch for split-K: -1 heuristic (default), 0 off, n > 1 that many
    splits wherever eligible."""
    load_kernels().vgpu_conv_set_splitk(mode)
    _WS_BYTES.clear()


def conv23(x: torch.Tensor, w2: torch.Tensor, b2: torch.Tensor, w3: torch.Tensor,
           residual: torch.Tensor, *, stride: int = 1, out: torch.Tensor | None = None) -> torch.Tensor:
    """Fused bottleneck tail: y = conv1x1(relu(conv3x3(x, w2, stride, pad 1) + b2), w3) + residual.

    x [N,W,H,Wd] with W ∈ {64, 128}; w2 [W,W,3,3]; b2 fp32 [W]; w3 [4W,W,1,1];
    residual [N,4W,OH,OW].  The conv2 activation stays on-chip (native/kernels/conv_gemm.hip,
    conv23_kernel); numerics equal conv2d(conv2d(...)) with the bf16 intermediate."""
    _nhwc(x, "x")
    _nhwc(w2, "w2")
    _nhwc(w3, "w3")
    _nhwc(residual, "residual")
    n, c, h, wd = x.shape
    if c not in (64, 128) or tuple(w2.shape) != (c, c, 3, 3) or tuple(w3.shape) != (4 * c, c, 1, 1):
        raise ValueError(f"unsupported fused conv2+conv3: x {tuple(x.shape)} w2 {tuple(w2.shape)} "
                         f"w3 {tuple(w3.shape)}")
    if b2.dtype != torch.float32 or not b2.is_contiguous() or b2.numel() != c:
        raise TypeError("b2 must be a contiguous fp32 tensor of size C")
    oh, ow = out_hw(h, wd, 3, stride, 1)
    if tuple(residual.shape) != (n, 4 * c, oh, ow):
        raise ValueError("residual shape")
    if out is None:
        out = torch.empty((n, 4 * c, oh, ow), dtype=x.dtype, device=x.device, memory_format=_CL)
    rc = load_kernels().vgpu_conv23_nhwc(_ptr(x), _ptr(w2), _ptr(b2), _ptr(w3), _ptr(residual), _ptr(out),
                                         n, h, wd, c, stride, _stream())
    if rc != 0:
        raise RuntimeError(f"vgpu_conv23_nhwc: error {rc}")
    return out


def conv231(x: torch.Tensor, w2: torch.Tensor, b2: torch.Tensor, w3: torch.Tensor,
            residual: torch.Tensor, w1n: torch.Tensor, b1n: torch.Tensor,
            pro_n: tuple[torch.Tensor, torch.Tensor], *, stride: int = 1) -> tuple[torch.Tensor, torch.Tensor]:
    """conv23 plus the next identity-shortcut block's conv1 in one kernel:
    y = conv23(x, ...) (the next block's input, still stored as its residual) and
    h1n = relu(conv1x1(relu(y*s + t), w1n) + b1n) with (s, t) = pro_n.  Numerics
    equal conv23 followed by conv2d(y, w1n, b1n, act='relu', pro=pro_n)."""
    _nhwc(x, "x")
    for t, nm in ((w2, "w2"), (w3, "w3"), (residual, "residual"), (w1n, "w1n")):
        _nhwc(t, nm)
    n, c, h, wd = x.shape
    if (c not in (64, 128) or tuple(w2.shape) != (c, c, 3, 3) or tuple(w3.shape) != (4 * c, c, 1, 1)
            or tuple(w1n.shape) != (c, 4 * c, 1, 1)):
        raise ValueError(f"unsupported fused tail + next conv1: x {tuple(x.shape)} w1n {tuple(w1n.shape)}")
    for p_, nm, size in ((b2, "b2", c), (b1n, "b1n", c), (pro_n[0], "scale", 4 * c), (pro_n[1], "shift", 4 * c)):
        if p_.dtype != torch.float32 or not p_.is_contiguous() or p_.numel() != size:
            raise TypeError(f"{nm} must be a contiguous fp32 tensor of size {size}")
    oh, ow = out_hw(h, wd, 3, stride, 1)
    if tuple(residual.shape) != (n, 4 * c, oh, ow):
        raise ValueError("residual shape")
    y = torch.empty((n, 4 * c, oh, ow), dtype=x.dtype, device=x.device, memory_format=_CL)
    h1 = torch.empty((n, c, oh, ow), dtype=x.dtype, device=x.device, memory_format=_CL)
    rc = load_kernels().vgpu_conv231_nhwc(_ptr(x), _ptr(w2), _ptr(b2), _ptr(w3), _ptr(residual), _ptr(y),
                                          _ptr(w1n), _ptr(b1n), _ptr(pro_n[0]), _ptr(pro_n[1]), _ptr(h1),
                                          n, h, wd, c, stride, _stream())
    if rc != 0:
        raise RuntimeError(f"vgpu_conv231_nhwc: error {rc}")
    return y, h1


def conv23_supported(c: int) -> bool:
    return c in (64, 128)


# ---- ResNet stem as a space-to-depth conv ------------------------------------------
# conv7x7/s2/p3 over C=3 == conv4x4/s1/p0 over X = s2d(pad(x)) with C = 12 (→16):
#   out[oh,ow] = Σ_{a,a',b,b',c} X[oh+a, ow+a', (b,b',c)] · W8[c, 2a+b, 2a'+b']
# (W8 = the 7x7 filter zero-padded to 8x8).  The MFMA conv then sees 16-B-aligned
# taps instead of 6-byte pixels.

def stem_s2d_shape(h: int, w: int, k: int = 7, stride: int = 2, pad: int = 3) -> tuple[int, int, int, int]:
    """(OH, OW, HS, WS) of a k×k/stride-2 stem and its space-to-depth input."""
    if stride != 2 or k % 2 != 1:
        raise ValueError("space-to-depth stem needs an odd kernel with stride 2")
    oh, ow = out_hw(h, w, k, stride, pad)
    kk = (k + 1) // 2
    return oh, ow, oh + kk - 1, ow + kk - 1


def stem_weight_s2d(w: torch.Tensor) -> torch.Tensor:
    """[Cout,3,k,k] (k odd) → [Cout,16,(k+1)/2,(k+1)/2] bf16 channels_last."""
    cout, c, k, _ = w.shape
    if c != 3 or k % 2 != 1:
        raise ValueError("stem weight must be [Cout,3,k,k] with k odd")
    kk = (k + 1) // 2
    w8 = torch.zeros(cout, c, 2 * kk, 2 * kk, dtype=torch.float32, device=w.device)
    w8[:, :, :k, :k] = w.float()
    # (o, c, a, b, a', b') → (o, a, a', b, b', c)
    t = w8.view(cout, c, kk, 2, kk, 2).permute(0, 2, 4, 3, 5, 1).reshape(cout, kk, kk, 4 * c)
    t = F.pad(t, (0, 16 - 4 * c))
    return t.to(w.dtype).permute(0, 3, 1, 2).contiguous(memory_format=_CL)


def stem_space_to_depth(x: torch.Tensor, k: int = 7, pad: int = 3) -> torch.Tensor:
    """x [N,3,H,W] bf16 channels_last → X [N,16,HS,WS] bf16 channels_last."""
    _nhwc(x, "x")
    n, c, h, w = x.shape
    if c != 3:
        raise ValueError("stem input must have 3 channels")
    _, _, hs, ws = stem_s2d_shape(h, w, k, 2, pad)
    out = torch.empty((n, 16, hs, ws), dtype=x.dtype, device=x.device, memory_format=_CL)
    rc = load_kernels().vgpu_stem_space_to_depth(_ptr(x), _ptr(out), n, h, w, pad, hs, ws, _stream())
    if rc != 0:
        raise RuntimeError(f"vgpu_stem_space_to_depth: error {rc}")
    return out


def stem_conv(x: torch.Tensor, w_s2d: torch.Tensor, k: int = 7, pad: int = 3) -> torch.Tensor:
    """7x7/s2 stem on the MFMA conv: space-to-depth + 4x4/s1 narrow-C conv."""
    return conv2d(stem_space_to_depth(x, k, pad), w_s2d)


def stem_pool(x: torch.Tensor, w_s2d: torch.Tensor, k: int = 7, pad: int = 3) -> torch.Tensor:
    """maxpool3s2(stem_conv(x, w_s2d)) in one kernel (the stem activation never
    reaches HBM); bit-identical to the two-kernel path, which it falls back to
    for shapes the fused kernel does not take (stem rows wider than 176)."""
    X = stem_space_to_depth(x, k, pad)
    n, _, hs, ws = X.shape
    if w_s2d.shape[0] != 64:
        return maxpool3s2(conv2d(X, w_s2d))
    oh, ow = hs - 3, ws - 3
    ph, pw = out_hw(oh, ow, 3, 2, 1)
    out = torch.empty((n, 64, ph, pw), dtype=x.dtype, device=x.device, memory_format=_CL)
    rc = load_kernels().vgpu_stem_pool_nhwc(_ptr(X), _ptr(w_s2d), _ptr(out), n, hs, ws, _stream())
    if rc == -1:
        return maxpool3s2(conv2d(X, w_s2d))
    if rc != 0:
        raise RuntimeError(f"vgpu_stem_pool_nhwc: error {rc}")
    return out


def maxpool(x: torch.Tensor, k: int, stride: int, pad: int = 0) -> torch.Tensor:
    """k×k max pool, NHWC bf16 (ResNet stem: 3/2/1; VGG: 2/2/0)."""
    _nhwc(x, "x")
    n, c, h, w = x.shape
    oh, ow = out_hw(h, w, k, stride, pad)
    out = torch.empty((n, c, oh, ow), dtype=x.dtype, device=x.device, memory_format=_CL)
    rc = load_kernels().vgpu_maxpool_nhwc(_ptr(x), _ptr(out), n, h, w, c, k, stride, pad, _stream())
    if rc != 0:
        raise RuntimeError(f"vgpu_maxpool_nhwc: error {rc}")
    return out


def maxpool3s2(x: torch.Tensor) -> torch.Tensor:
    return maxpool(x, 3, 2, 1)


class _MaxPoolTrainFn(torch.autograd.Function):
    """k×k max pool with a one-byte winning-tap index per output element
    (native/kernels/pool_train.hip); backward gathers dy per input pixel."""

    @staticmethod
    def forward(ctx, x, k: int, stride: int, pad: int):
        n, c, h, w = x.shape
        oh, ow = out_hw(h, w, k, stride, pad)
        y = torch.empty((n, c, oh, ow), dtype=x.dtype, device=x.device, memory_format=_CL)
        idx = torch.empty((n, oh, ow, c), dtype=torch.uint8, device=x.device)
        rc = load_kernels().vgpu_maxpool_fwd_idx_nhwc(_ptr(x), _ptr(y), _ptr(idx), n, h, w, c, k, stride, pad,
                                                     _stream())
        if rc != 0:
            raise RuntimeError(f"vgpu_maxpool_fwd_idx_nhwc: error {rc}")
        ctx.save_for_backward(idx)
        ctx.cfg = (n, c, h, w, k, stride, pad)
        ctx.mark_non_differentiable(idx)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        n, c, h, w, k, stride, pad = ctx.cfg
        dy = dy.contiguous(memory_format=_CL)
        dx = torch.empty((n, c, h, w), dtype=dy.dtype, device=dy.device, memory_format=_CL)
        rc = load_kernels().vgpu_maxpool_bwd_nhwc(_ptr(dy), _ptr(idx), _ptr(dx), n, h, w, c, k, stride, pad,
                                                 _stream())
        if rc != 0:
            raise RuntimeError(f"vgpu_maxpool_bwd_nhwc: error {rc}")
        return dx, None, None, None


def maxpool_train(x: torch.Tensor, pool: torch.nn.MaxPool2d) -> torch.Tensor:
    """pool(x) with the native forward / backward for bf16 channels_last CUDA
    tensors (square window, no dilation, no ceil mode), else the module."""
    k, s, p = pool.kernel_size, pool.stride, pool.padding
    k = k if isinstance(k, int) else (k[0] if k[0] == k[1] else None)
    s = s if isinstance(s, int) else (s[0] if s[0] == s[1] else None)
    p = p if isinstance(p, int) else (p[0] if p[0] == p[1] else None)
    if (not _TRAIN_NATIVE or k is None or s is None or p is None or pool.ceil_mode or pool.dilation not in (1, (1, 1))
            or pool.return_indices or not x.is_cuda or x.dtype != torch.bfloat16 or x.dim() != 4
            or not x.is_contiguous(memory_format=_CL) or x.shape[1] % 8 or 2 * p > k):
        return pool(x)
    return _MaxPoolTrainFn.apply(x, k, s, p)


def scale_shift_relu_mean(x: torch.Tensor, scale: torch.Tensor, shift: torch.Tensor) -> torch.Tensor:
    """mean over H,W of relu(x*scale[c] + shift[c]) → [N, C] bf16 (final BN+ReLU+pool)."""
    _nhwc(x, "x")
    n, c, h, w = x.shape
    out = torch.empty((n, c), dtype=x.dtype, device=x.device)
    rc = load_kernels().vgpu_scale_shift_relu_mean_nhwc(_ptr(x), _ptr(scale), _ptr(shift), _ptr(out),
                                                       n, h * w, c, _stream())
    if rc != 0:
        raise RuntimeError(f"vgpu_scale_shift_relu_mean_nhwc: error {rc}")
    return out


# ---- training: native forward / data gradient, MIOpen weight gradient -------------------
# VGPU_NATIVE_CONV_TRAIN=0 keeps every training convolution on MIOpen (A/B).
_TRAIN_NATIVE = os.environ.get("VGPU_NATIVE_CONV_TRAIN", "1") != "0"


def conv2d_wgrad(dy: torch.Tensor, x: torch.Tensor, ks: int, *, stride: int = 1,
                 padding: int = 0, db_job: tuple | None = None) -> torch.Tensor:
    """Weight gradient of y = conv2d(x, w, stride, padding) for a [Cout, C, ks, ks]
    channels_last bf16 weight, on the MFMA kernel (native/kernels/conv_wgrad.hip:
    split-K over output pixels, fp32 partials, deterministic reduce).
    dy [N,Cout,OH,OW] and x [N,C,H,W] bf16 channels_last; C, Cout multiples of 64."""
    _nhwc(dy, "dy")
    _nhwc(x, "x")
    n, c, h, wd = x.shape
    cout = dy.shape[1]
    if c % 64 or cout % 64 or dy.shape[0] != n or tuple(dy.shape[2:]) != out_hw(h, wd, ks, stride, padding):
        raise ValueError(f"unsupported wgrad: dy {tuple(dy.shape)} x {tuple(x.shape)} ks {ks}")
    lib = load_kernels()
    need = lib.vgpu_conv_wgrad_workspace(n, h, wd, c, cout, ks, stride, padding)
    if need < 0:
        raise ValueError("unsupported wgrad shape")
    ws = torch.empty(max(need // 4, 1), dtype=torch.float32, device=x.device)
    dw = torch.empty((cout, c, ks, ks), dtype=x.dtype, device=x.device, memory_format=_CL)
    if db_job is not None:  # (partials, slabs, db, stride): the bias gradient summed in the same reduce launch
        part, slabs, db, pst = db_job
        rc = lib.vgpu_conv_wgrad_db_nhwc(_ptr(dy), _ptr(x), _ptr(dw), _ptr(ws), need, n, h, wd, c, cout, ks, stride,
                                         padding, _ptr(part), slabs, db.numel(), _ptr(db),
                                         int(db.dtype == torch.bfloat16), pst, _stream())
    else:
        rc = lib.vgpu_conv_wgrad_nhwc(_ptr(dy), _ptr(x), _ptr(dw), _ptr(ws), need, n, h, wd, c, cout,
                                      ks, stride, padding, _stream())
    if rc != 0:
        raise RuntimeError(f"vgpu_conv_wgrad_nhwc: error {rc}")
    return dw


# Weight gradient in training: the native kernel where it measured ahead of
# MIOpen: every 1x1 convolution, and 3x3 over ≥ 8k output pixels (tap-fused
# kernel on stage 1, per-tap GEMMs after); profiles/wgrad_r1.md, profiles/r4/train.
# MIOpen elsewhere.  VGPU_CONV_WGRAD=0: always MIOpen; =all: always native.
_WGRAD_MODE = os.environ.get("VGPU_CONV_WGRAD", "auto")


def _wgrad_native(dy: torch.Tensor, ks: int, stride: int, c: int = 0) -> bool:
    if _WGRAD_MODE == "0":
        return False
    if _WGRAD_MODE == "all":
        return True
    pixels = dy.shape[0] * dy.shape[2] * dy.shape[3]
    # 1x1 (stride 1 or 2) from 1k output pixels: the swizzled LDS images run
    # 23-36 us vs MIOpen's 27-43 us plus its zero-fill and cast passes
    # (profiles/r4/train/convtrain_wgrad_swizzle.log); at ResNet-V2-152's
    # stage 4 (640 pixels) MIOpen's kernel measured ahead in eager timing
    # (16-20 vs 24-33 us, convtrain_b10_256.log).
    # Round 5, timed inside hipGraph replays (the training steps are replays;
    # the round-4 thresholds came from eager timings with a ~11 us launch floor):
    # every 3x3 shape measured runs faster natively -- VGG-16 b=2 at 392 / 1568
    # pixels 12.8 / 31-51 us vs MIOpen's 42 / 69-82 us, ResNet-V2-152 b=10 stage
    # 3 / 4 26.6 / 41.8 vs 62 / 53, ResNet-V2-50 stage 4 (2.4k pixels) 59 vs 82
    # (profiles/r5/train/vgg_small_ab*.log: MIOpen's kernel plus its zero-fill
    # and cast passes).
    # Round 6: 1x1 at any size.  DeepLab-v3 4.2 (b=1) has 40 1x1 layers on
    # 576-pixel maps; MIOpen's weight gradient there is its kernel plus a
    # zero-fill and a cast pass (3 dispatches of ~5 us inside a replayed step,
    # 180 of the step's 790, profiles/r6/train), the native one 1-2.
    if ks == 1:
        return pixels >= 1
    return ks == 3


# ---- data-gradient filters, one launch per step ------------------------------------------
# id(weight) -> (transposed + flipped filter, weight._version it was built from, data_ptr)
_DGRAD: dict[int, tuple[torch.Tensor, int, int]] = {}  # + the weight's data_ptr


class DgradFilters:
    """The transposed, flipped filters the data gradient of every stride-1
    training conv of a model needs, rebuilt by ONE batched kernel
    (native/kernels/weights.hip) instead of a transpose + flip + copy per layer
    and step (~100 small kernels, 380 us of a ResNet-V2-50 step).  Call
    refresh() at the start of each training forward; _ConvTrainFn's backward
    takes a filter from here when the weight has not changed since."""

    def __init__(self, convs):
        self._all = list(convs)
        self._build()

    def _build(self):
        import struct
        convs = self._all
        # stride-1 convs (their data gradient is a conv with this filter) and 1x1
        # projection shortcuts of any stride (a 1x1 GEMM on the compact grid)
        self.convs = [c for c in convs if (c.stride == (1, 1) or c.kernel_size == (1, 1))
                      and c.kernel_size[0] in (1, 3)
                      and c.weight.is_cuda and c.weight.dtype == torch.bfloat16
                      and c.weight.is_contiguous(memory_format=_CL) and c.groups == 1
                      and c.in_channels % 64 == 0 and c.out_channels % 64 == 0]
        self.bufs = []
        if not self.convs:
            self.desc = None
            return
        lib = load_kernels()
        if lib.vgpu_wt_desc_size() != 32:
            raise RuntimeError("weights.hip descriptor layout changed")
        raw, tile0 = b"", 0
        for c in self.convs:
            w = c.weight
            ks = c.kernel_size[0]
            wt = torch.empty((c.in_channels, c.out_channels, ks, ks), dtype=w.dtype, device=w.device,
                             memory_format=_CL)
            self.bufs.append(wt)
            raw += struct.pack("<QQiiii", w.data_ptr(), wt.data_ptr(), c.out_channels, c.in_channels, ks, tile0)
            tile0 += lib.vgpu_wt_flip_tiles(c.out_channels, c.in_channels, ks)
        self.tiles = tile0
        self.ptrs = [c.weight.data_ptr() for c in self.convs]
        self.desc = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.convs[0].weight.device)

    def refresh(self) -> None:
        if self.desc is None:
            return
        # The table holds raw weight addresses: a weight re-allocated since
        # (model.to(...), load_state_dict with assign=True) would be read from
        # freed memory, so rebuild first.
        if any(c.weight.data_ptr() != p for c, p in zip(self.convs, self.ptrs)):
            self._build()
            if self.desc is None:
                return
        rc = load_kernels().vgpu_wt_flip_batched(_ptr(self.desc), len(self.convs), self.tiles, _stream())
        if rc != 0:
            raise RuntimeError(f"vgpu_wt_flip_batched: error {rc}")
        for c, wt in zip(self.convs, self.bufs):
            _DGRAD[id(c.weight)] = (wt, c.weight._version, c.weight.data_ptr())


def _dgrad_filter(w: torch.Tensor) -> torch.Tensor:
    hit = _DGRAD.get(id(w))
    if hit is not None and hit[1] == w._version and hit[2] == w.data_ptr() and hit[0].shape[0] == w.shape[1]:
        return hit[0]
    ks = w.shape[2]
    wt = w.transpose(0, 1)
    if ks > 1:
        wt = wt.flip(2, 3)
    return wt.contiguous(memory_format=_CL)


class _ConvTrainFn(torch.autograd.Function):
    """y = conv(x, w) (+ residual) on the MFMA kernel; backward: dx on the same
    kernel (stride 1: the data gradient is a stride-1 convolution of dy with the
    transposed, spatially flipped filter and padding k-1-p), dw on the native
    weight-gradient kernel where it wins (_wgrad_native), else MIOpen.
    Per-layer timings that motivated the split: profiles/convtrain_r1.md."""

    @staticmethod
    def forward(ctx, x, w, residual, stride: int, padding: int, res_out: bool = False):
        y = conv2d(x, w, stride=stride, padding=padding, residual=residual)
        ctx.save_for_backward(x, w)
        ctx.stride, ctx.padding = stride, padding
        ctx.has_res = residual is not None
        ctx.set_materialize_grads(False)
        if res_out:
            # x again as an output: the gradient it receives (an identity
            # shortcut's) is added by the data-gradient kernel's epilogue instead
            # of an autograd accumulation pass over x
            return y, x.view_as(x)
        return y

    @staticmethod
    def backward(ctx, dy, dxres=None):
        x, w = ctx.saved_tensors
        if dy is None:  # only the shortcut output was used
            return dxres, None, None, None, None, None
        dy = dy.contiguous(memory_format=_CL)
        dx, dw = conv_backward(dy, x, w, ctx.stride, ctx.padding, ctx.needs_input_grad[0], ctx.needs_input_grad[1],
                               dx_add=dxres)
        dres = dy if ctx.has_res and ctx.needs_input_grad[2] else None
        return dx, dw, dres, None, None, None


def conv_backward(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor, s: int, p: int, need_dx: bool,
                  need_dw: bool, *, skip_dx: bool = False, db_job: tuple | None = None,
                  dx_add: torch.Tensor | None = None) -> tuple[torch.Tensor | None, torch.Tensor | None]:
    """(dx, dw) of y = conv(x, w, stride s, padding p): dx on the MFMA kernel for
    stride 1 (MIOpen otherwise), dw per _wgrad_native.  skip_dx: the caller
    computed a stride-1 dx itself (vgpu.ops.bnconv's fused data gradient).
    dx_add: a second gradient of x, summed into dx (in the kernel's epilogue
    for stride 1)."""
    common = ([0], [s, s], [p, p], [1, 1], False, [0, 0], 1)
    bw = torch.ops.aten.convolution_backward
    dx = dw = None
    native_dw = need_dw and _wgrad_native(dy, w.shape[2], s, w.shape[1])
    if s == 1:
        if need_dx and not skip_dx:
            ks = w.shape[2]
            add = dx_add.contiguous(memory_format=_CL) if dx_add is not None else None
            dx = conv2d(dy, _dgrad_filter(w), stride=1, padding=ks - 1 - p, residual=add)
            dx_add = None
    elif need_dx:
        dx, dw, _ = bw(dy, x, w, *common, [True, need_dw and not native_dw, False])
    if dx_add is not None and dx is not None:
        dx = dx + dx_add
    if native_dw:
        dw = conv2d_wgrad(dy, x, w.shape[2], stride=s, padding=p, db_job=db_job)
        db_job = None
    elif need_dw and dw is None:
        dw = bw(dy, x, w, *common, [False, True, False])[1]
    if db_job is not None:  # no native weight-gradient reduce to ride along with
        part, slabs, db, pst = db_job
        rc = load_kernels().vgpu_bias_grad_reduce(_ptr(part), slabs, db.numel(), _ptr(db),
                                                  int(db.dtype == torch.bfloat16), pst, _stream())
        if rc != 0:
            raise RuntimeError(f"vgpu_bias_grad_reduce: error {rc}")
    return dx, dw


def native_train_enabled() -> bool:
    return _TRAIN_NATIVE


def train_eligible(x: torch.Tensor, conv: torch.nn.Conv2d) -> bool:
    w = conv.weight
    return (_TRAIN_NATIVE and x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and x.dim() == 4 and x.is_contiguous(memory_format=_CL) and w.is_contiguous(memory_format=_CL)
            and conv.bias is None and conv.groups == 1 and conv.dilation == (1, 1)
            and conv.kernel_size[0] == conv.kernel_size[1] and conv.stride[0] == conv.stride[1]
            and conv.padding[0] == conv.padding[1] and isinstance(conv.padding[0], int)
            and supported(conv.in_channels, conv.out_channels, conv.kernel_size[0])
            and conv.kernel_size[0] in (1, 3))


def conv_train(x: torch.Tensor, conv: torch.nn.Conv2d, residual: torch.Tensor | None = None,
               res_out: bool = False):
    """conv(x) (+ residual) with the module's semantics; bf16 channels_last CUDA
    tensors of supported shapes run natively, anything else through the module.
    res_out: return (y, x') where x' is x for use as an identity shortcut, whose
    gradient the data-gradient kernel then sums into dx."""
    if not train_eligible(x, conv) or (residual is not None and not residual.is_contiguous(memory_format=_CL)):
        y = conv(x)
        y = y if residual is None else y + residual
        return (y, x) if res_out else y
    return _ConvTrainFn.apply(x, conv.weight, residual, conv.stride[0], conv.padding[0], res_out)


class _ConvBiasReLUTrainFn(torch.autograd.Function):
    """y = relu(conv(x, w) + b) in one MFMA kernel pass (bias + ReLU in the
    epilogue).  Backward: g = dy masked by y > 0 (one threshold pass), db =
    Σ g in fp32, then dx / dw exactly as _ConvTrainFn (conv_backward).  The
    VGG-16 training path (vgpu.models.vision.VGG16)."""

    @staticmethod
    def forward(ctx, x, w, b, stride: int, padding: int, in_relu: bool = False):
        y = conv2d(x, w, b, stride=stride, padding=padding, act="relu")
        ctx.save_for_backward(x, w, y)
        ctx.bias_dtype = b.dtype
        ctx.stride, ctx.padding, ctx.in_relu = stride, padding, in_relu
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        link = _RELU_LINK.pop(dy.data_ptr(), None)
        if link is not None and link[0] == "mask" and dy.is_contiguous(memory_format=_CL):
            # the next layer's data gradient already applied this layer's ReLU mask
            # and summed its bias-gradient partials (dgrad_into_relu)
            g, (_, part, slabs, pst) = dy, link
        else:
            g, part, slabs = relu_bias_grad_partial(dy.contiguous(memory_format=_CL), y)
            pst = 1
        db = torch.empty(y.shape[1], dtype=ctx.bias_dtype, device=y.device) if ctx.needs_input_grad[2] else None
        dx, dw = _backward_into(ctx, g, x, w, (part, slabs, db, pst) if db is not None else None)
        return dx, dw, db, None, None, None


# data_ptr of a gradient already masked for its ReLU layer -> (partials, count,
# stride) of that layer's bias gradient: dgrad_into_relu hands them from one
# conv + ReLU layer's backward to the previous layer's (VGG16._train_features
# clears it each forward; an entry nobody pops is just dropped then).
_RELU_LINK: dict[int, tuple] = {}
_RELU_COEF: dict[tuple, torch.Tensor] = {}
# data_ptr of a fused conv + ReLU + pool block's output -> (argmax, ReLU output,
# k, weakref to that output).  Used only for a consumer told (in_relu == 2) that
# the block's output feeds it alone: its x-gradient is then never formed.
_POOL_SRC: dict[int, tuple] = {}


def dgrad_into_pool(dy: torch.Tensor, w: torch.Tensor, padding: int, idx: torch.Tensor, yfull: torch.Tensor, k: int):
    """Stride-1 data gradient of conv(x, w) where x = maxpool_k(yfull) and yfull
    a ReLU output: scattered through the pool's argmax into yfull's resolution,
    masked by yfull > 0, with the bias partials of yfull's layer -- (g_full,
    partials, count) -- or None unless the conv runs split-K."""
    ks = w.shape[2]
    wf = _dgrad_filter(w)
    n, c, h, wd = dy.shape
    cout = wf.shape[0]
    p2 = ks - 1 - padding
    oh, ow = out_hw(h, wd, ks, 1, p2)
    if (tuple(idx.shape) != (n, oh, ow, cout) or tuple(yfull.shape) != (n, cout, oh * k, ow * k)
            or not yfull.is_contiguous(memory_format=_CL) or 256 % (cout // 8)):
        return None
    lib = load_kernels()
    need = lib.vgpu_conv2d_workspace(n, h, wd, c, cout, ks, 1, p2, 0)
    if need <= 0:
        return None
    blocks = (n * oh * ow * (cout // 8) + 255) // 256
    gpart = torch.empty(blocks * cout, dtype=torch.float32, device=dy.device)
    ws = torch.empty(need // 4, dtype=torch.float32, device=dy.device)
    g = torch.empty_like(yfull, memory_format=_CL)
    nb = ctypes.c_int(0)
    rc = lib.vgpu_conv2d_masked_pool_splitk(_ptr(dy), _ptr(wf), n, h, wd, c, cout, ks, p2, _ptr(idx), k, _ptr(yfull),
                                            _ptr(g), _ptr(gpart), gpart.numel() * 4, _ptr(ws), need,
                                            ctypes.byref(nb), _stream())
    if rc == -1:
        return None
    if rc != 0:
        raise RuntimeError(f"vgpu_conv2d_masked_pool_splitk: error {rc}")
    return g, gpart, nb.value


def _relu_coef(c: int, device) -> torch.Tensor:
    """BN coefficients (s, t, mean, invstd) = (1, 0, 0, 1): the statistics
    epilogue then masks by x > 0 and sums (Σv, Σv·x)."""
    key = (c, str(device))
    t = _RELU_COEF.get(key)
    if t is None:
        t = torch.zeros((4, c), dtype=torch.float32, device=device)
        t[0] = 1.0
        t[3] = 1.0
        _RELU_COEF[key] = t
    return t


def dgrad_into_relu(dy: torch.Tensor, w: torch.Tensor, padding: int, mask: torch.Tensor):
    """Stride-1 data gradient of conv(x, w) masked by [mask > 0] -- the ReLU of
    the layer that produced x (mask = x) -- plus that layer's bias-gradient
    partial sums: (g, partials, count, stride) or None when no fused kernel
    takes the shape.  Split-K shapes mask in the split reduce; the others use
    the BatchNorm-statistics epilogue with unit coefficients (Σ v per 64 rows)."""
    ks = w.shape[2]
    wf = _dgrad_filter(w)
    n, c, h, wd = dy.shape
    cout = wf.shape[0]
    p2 = ks - 1 - padding
    oh, ow = out_hw(h, wd, ks, 1, p2)
    if (n, cout, oh, ow) != tuple(mask.shape) or not mask.is_contiguous(memory_format=_CL):
        return None
    lib = load_kernels()
    out = torch.empty((n, cout, oh, ow), dtype=dy.dtype, device=dy.device, memory_format=_CL)
    need = lib.vgpu_conv2d_workspace(n, h, wd, c, cout, ks, 1, p2, 0)
    m = n * oh * ow
    if need > 0 and 256 % (cout // 8) == 0:
        blocks = (m * (cout // 8) + 255) // 256
        gpart = torch.empty(blocks * cout, dtype=torch.float32, device=dy.device)
        ws = torch.empty(need // 4, dtype=torch.float32, device=dy.device)
        nb = ctypes.c_int(0)
        rc = lib.vgpu_conv2d_masked_splitk(_ptr(dy), _ptr(wf), _ptr(out), n, h, wd, c, cout, ks, p2, _ptr(mask),
                                           _ptr(gpart), gpart.numel() * 4, _ptr(ws), need, ctypes.byref(nb),
                                           _stream())
        if rc == 0:
            return out, gpart, nb.value, 1
        if rc != -1:
            raise RuntimeError(f"vgpu_conv2d_masked_splitk: error {rc}")
        return None
    groups = (m + 63) // 64
    stats = torch.empty(groups * cout * 2, dtype=torch.float32, device=dy.device)
    rc = lib.vgpu_conv2d_nhwc_bn(_ptr(dy), _ptr(wf), _ptr(out), None, n, h, wd, c, cout, ks, 1, p2, _ptr(stats),
                                 _ptr(mask), _ptr(_relu_coef(cout, dy.device)), 1, 1, _stream())
    if rc == 0:
        return out, stats, groups, 2
    if rc != -1:
        raise RuntimeError(f"vgpu_conv2d_nhwc_bn: error {rc}")
    return None


def _backward_into(ctx, g, x, w, db_job):
    """dx, dw of a conv + ReLU layer from its masked gradient g.  When the
    layer's input is itself a ReLU output (ctx.in_relu), dx comes out masked for
    that layer with its bias partials linked for its backward."""
    need_dx, need_dw = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
    if need_dx and ctx.in_relu == 1 and ctx.stride == 1:
        fused = dgrad_into_relu(g, w, ctx.padding, x)
        if fused is not None:
            dx, part, count, pst = fused
            _RELU_LINK[dx.data_ptr()] = ("mask", part, count, pst)
            _, dw = conv_backward(g, x, w, 1, ctx.padding, True, need_dw, skip_dx=True, db_job=db_job)
            return dx, dw
    src = _POOL_SRC.get(x.data_ptr()) if need_dx and ctx.in_relu == 2 and ctx.stride == 1 else None
    if src is not None and src[3]() is not None and src[3]().data_ptr() == x.data_ptr():
        fused = dgrad_into_pool(g, w, ctx.padding, *src[:3])
        if fused is not None:
            gfull, part, count = fused
            # x's gradient proper is never formed: the pool block's backward takes
            # gfull through the link (x feeds this conv only)
            dx = torch.empty_like(x, memory_format=_CL)
            _RELU_LINK[dx.data_ptr()] = ("pool", gfull, part, count)
            _, dw = conv_backward(g, x, w, 1, ctx.padding, True, need_dw, skip_dx=True, db_job=db_job)
            return dx, dw
    return conv_backward(g, x, w, ctx.stride, ctx.padding, need_dx, need_dw, db_job=db_job)


def relu_bias_grad_partial(dy: torch.Tensor, y: torch.Tensor, idx: torch.Tensor | None = None,
                           k: int = 0, dy_nchw: bool = False) -> tuple[torch.Tensor, torch.Tensor, int]:
    """(g, partials, slabs): g = dy·[y > 0] (dy arriving through a k×k / stride-k
    max pool with argmax idx when k > 0) and the per-slab column sums of g, fp32
    [slabs, C] -- the bias gradient is summed by the weight gradient's reduce
    launch (conv_backward's db_job).  dy_nchw: the pooled dy is NCHW-contiguous."""
    if dy_nchw:
        if not (k > 0 and dy.is_cuda and dy.dtype == torch.bfloat16 and dy.is_contiguous()):
            raise ValueError("dy_nchw needs a pooled, contiguous bf16 dy")
    else:
        _nhwc(dy, "dy")
    _nhwc(y, "y")
    n, c, h, w = y.shape
    lib = load_kernels()
    g = torch.empty_like(y, memory_format=_CL)
    need = lib.vgpu_relu_bias_grad_workspace(n * h * w, c)
    if need < 0:
        raise ValueError("unsupported relu_bias_grad shape")
    part = torch.empty(max(need // 4, 1), dtype=torch.float32, device=y.device)
    slabs = ctypes.c_int(0)
    rc = lib.vgpu_relu_bias_grad_partial2(_ptr(dy), _ptr(idx), _ptr(y), _ptr(g), _ptr(part), n, h, w, c, k,
                                          int(dy_nchw), ctypes.byref(slabs), _stream())
    if rc != 0:
        raise RuntimeError(f"vgpu_relu_bias_grad_partial2: error {rc}")
    return g, part, slabs.value


def relu_bias_grad(dy: torch.Tensor, y: torch.Tensor,
                   db_dtype: torch.dtype = torch.float32) -> tuple[torch.Tensor, torch.Tensor]:
    """(g, db): g = dy where y > 0 else 0 (bf16, channels_last), db = Σ g over
    N, H, W summed in fp32 and stored as db_dtype (fp32 or the bias's bf16) --
    one pass (native/kernels/fused_eltwise.hip)."""
    _nhwc(dy, "dy")
    _nhwc(y, "y")
    n, c, h, w = y.shape
    rows = n * h * w
    lib = load_kernels()
    g = torch.empty_like(y, memory_format=_CL)
    if db_dtype not in (torch.float32, torch.bfloat16):
        raise TypeError(db_dtype)
    db = torch.empty(c, dtype=db_dtype, device=y.device)
    ws = torch.empty(max(lib.vgpu_relu_bias_grad_workspace(rows, c) // 4, 1), dtype=torch.float32, device=y.device)
    rc = lib.vgpu_relu_bias_grad_nhwc(_ptr(dy), _ptr(y), _ptr(g), _ptr(db), _ptr(ws), rows, c,
                                      int(db_dtype == torch.bfloat16), _stream())
    if rc != 0:
        raise RuntimeError(f"vgpu_relu_bias_grad_nhwc: error {rc}")
    return g, db


class _ConvBiasReLUPoolTrainFn(torch.autograd.Function):
    """maxpool_k×k/stride k(relu(conv(x, w) + b)): the conv with bias + ReLU
    in its epilogue, then the pool with its one-byte argmax.  Backward: the
    pool's gradient gather, the ReLU mask and the bias gradient in ONE pass
    (vgpu_pool_relu_bias_grad_nhwc), then dx / dw as _ConvTrainFn.  VGG-16's
    five conv + ReLU + pool blocks."""

    @staticmethod
    def forward(ctx, x, w, b, stride: int, padding: int, k: int, in_relu: bool = False, out_nchw: bool = False):
        ctx.in_relu, ctx.out_nchw = in_relu, out_nchw
        y = conv2d(x, w, b, stride=stride, padding=padding, act="relu")
        n, c, h, wd = y.shape
        oh, ow = h // k, wd // k
        idx = torch.empty((n, oh, ow, c), dtype=torch.uint8, device=y.device)
        if out_nchw:  # a flatten follows: NCHW output makes it a view, no copy either way
            p = torch.empty((n, c, oh, ow), dtype=y.dtype, device=y.device)
            fn = load_kernels().vgpu_maxpool_fwd_idx_nchw_out
        else:
            p = torch.empty((n, c, oh, ow), dtype=y.dtype, device=y.device, memory_format=_CL)
            fn = load_kernels().vgpu_maxpool_fwd_idx_nhwc
        rc = fn(_ptr(y), _ptr(p), _ptr(idx), n, h, wd, c, k, k, 0, _stream())
        if rc != 0:
            raise RuntimeError(f"maxpool forward: error {rc}")
        ctx.save_for_backward(x, w, y, idx)
        ctx.mark_non_differentiable(idx)
        ctx.stride, ctx.padding, ctx.k, ctx.bias_dtype = stride, padding, k, b.dtype
        _POOL_SRC[p.data_ptr()] = (idx, y, k, weakref.ref(p))  # for the next conv's fused data gradient
        return p

    @staticmethod
    def backward(ctx, dp):
        x, w, y, idx = ctx.saved_tensors
        link = _RELU_LINK.pop(dp.data_ptr(), None)
        if link is not None and link[0] == "pool":
            # the next conv's split data gradient scattered through this pool,
            # masked by this ReLU and summed the bias partials (dgrad_into_pool);
            # dp itself was never written
            _, g, part, slabs = link
        elif ctx.out_nchw:
            g, part, slabs = relu_bias_grad_partial(dp.contiguous(), y, idx=idx, k=ctx.k, dy_nchw=True)
        else:
            dp = dp.contiguous(memory_format=_CL)
            g, part, slabs = relu_bias_grad_partial(dp, y, idx=idx, k=ctx.k)
        db = torch.empty(y.shape[1], dtype=ctx.bias_dtype, device=y.device) if ctx.needs_input_grad[2] else None
        dx, dw = _backward_into(ctx, g, x, w, (part, slabs, db, 1) if db is not None else None)
        return dx, dw, db, None, None, None, None, None


def conv_bias_relu_pool_train(x: torch.Tensor, conv: torch.nn.Conv2d, pool: torch.nn.MaxPool2d,
                              in_relu: int = 0, out_nchw: bool = False) -> torch.Tensor:
    """pool(relu(conv(x))) with the module semantics; the fused native path for
    a k×k / stride-k unpadded pool after a native-eligible conv, else the
    unfused ops."""
    k, s_, p_ = pool.kernel_size, pool.stride, pool.padding
    k = k if isinstance(k, int) else (k[0] if k[0] == k[1] else None)
    s_ = s_ if isinstance(s_, int) else (s_[0] if s_[0] == s_[1] else None)
    p_ = p_ if isinstance(p_, int) else (p_[0] if p_[0] == p_[1] else -1)
    w = conv.weight
    ok = (k is not None and s_ == k and p_ == 0 and not pool.ceil_mode and pool.dilation in (1, (1, 1))
          and not pool.return_indices and _conv_bias_relu_ok(x, conv)
          and conv.out_channels % 8 == 0 and conv.out_channels <= 2048 and w.dtype == torch.bfloat16)
    if not ok:
        return maxpool_train(conv_bias_relu_train(x, conv).contiguous(memory_format=_CL), pool)
    return _ConvBiasReLUPoolTrainFn.apply(x, w, conv.bias, conv.stride[0], conv.padding[0], k, in_relu, out_nchw)


def _conv_bias_relu_ok(x: torch.Tensor, conv: torch.nn.Conv2d) -> bool:
    w = conv.weight
    return (_TRAIN_NATIVE and conv.bias is not None and x.is_cuda and x.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and x.dim() == 4 and x.is_contiguous(memory_format=_CL)
            and w.is_contiguous(memory_format=_CL) and conv.groups == 1 and conv.dilation == (1, 1)
            and conv.kernel_size[0] == conv.kernel_size[1] and conv.stride[0] == conv.stride[1]
            and conv.padding[0] == conv.padding[1] and isinstance(conv.padding[0], int)
            and conv.kernel_size[0] in (1, 3) and supported(conv.in_channels, conv.out_channels, conv.kernel_size[0]))


class _PadChannelsFn(torch.autograd.Function):
    """Zero channels appended to an NHWC bf16 tensor in one kernel pass;
    the gradient is the leading-channel slice."""

    @staticmethod
    def forward(ctx, x, cp: int):
        n, c, h, w = x.shape
        y = torch.empty((n, cp, h, w), dtype=x.dtype, device=x.device, memory_format=_CL)
        rc = load_kernels().vgpu_pad_channels(_ptr(x), _ptr(y), n * h * w, c, cp, _stream())
        if rc != 0:
            raise RuntimeError(f"vgpu_pad_channels: error {rc}")
        ctx.c = c
        return y

    @staticmethod
    def backward(ctx, dy):
        return dy[:, :ctx.c].contiguous(memory_format=_CL), None


def pad_channels(x: torch.Tensor, cp: int) -> torch.Tensor:
    """x [N, C, H, W] bf16 channels_last → [N, cp, H, W] with zero channels C..cp-1."""
    _nhwc(x, "x")
    return _PadChannelsFn.apply(x, cp)


def conv_bias_relu_train(x: torch.Tensor, conv: torch.nn.Conv2d, in_relu: int = 0) -> torch.Tensor:
    """relu(conv(x)) with the module's semantics (bias included); bf16
    channels_last CUDA tensors of supported shapes run natively, anything else
    through the module.  in_relu: 1 when x is the previous conv + ReLU's output
    and feeds only this conv, 2 when x is a fused conv + ReLU + pool block's
    output and feeds only this conv -- the data gradient then does that layer's
    ReLU (and pool) backward (dgrad_into_relu / dgrad_into_pool)."""
    w = conv.weight
    c = conv.in_channels
    if (0 < c < 64 and conv.out_channels % 64 == 0 and _TRAIN_NATIVE and conv.bias is not None and x.is_cuda
            and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dim() == 4 and conv.groups == 1
            and conv.kernel_size == (3, 3) and conv.stride == (1, 1) and conv.padding == (1, 1)
            and conv.dilation == (1, 1)):
        # A narrow input (VGG's 3-channel first layer): zero channels up to 64
        # (differentiable pads, so the gradients slice back) and run the MFMA
        # conv and native weight gradient -- ~21x the MACs of the 3 real
        # channels, still far less time than MIOpen's two kernels at 224²
        # (prof_3_2.md: 49 us each).
        xp = pad_channels(x.contiguous(memory_format=_CL), 64)
        wp = pad_channels(w.contiguous(memory_format=_CL), 64)
        return _ConvBiasReLUTrainFn.apply(xp, wp, conv.bias, 1, 1)
    if not _conv_bias_relu_ok(x, conv):
        return F.relu(conv(x))
    return _ConvBiasReLUTrainFn.apply(x, w, conv.bias, conv.stride[0], conv.padding[0], in_relu)


# ---- fp32 references -----------------------------------------------------------------
def conv2d_ref(x, w, bias=None, *, stride=1, padding=0, act="none", pro=None, residual=None):
    xf = x.float()
    if pro is not None:
        xf = (xf * pro[0].view(1, -1, 1, 1) + pro[1].view(1, -1, 1, 1)).clamp_min(0)
        xf = xf.to(x.dtype).float()  # the kernel stages the prologue output as bf16
    y = F.conv2d(xf, w.float(), None if bias is None else bias.float(), stride=stride, padding=padding)
    if residual is not None:
        y = y + residual.float()
    if act == "relu":
        y = y.clamp_min(0)
    elif act == "relu6":
        y = y.clamp(0, 6)
    return y


def maxpool_ref(x, k, stride, pad=0):
    return F.max_pool2d(x.float(), k, stride, pad)


def scale_shift_relu_mean_ref(x, scale, shift):
    y = (x.float() * scale.view(1, -1, 1, 1) + shift.view(1, -1, 1, 1)).clamp_min(0)
    return y.mean(dim=(2, 3))
