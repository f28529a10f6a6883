"""VGG-16 and DeepLab-v3 (MobileNet-V2 backbone + ASPP) for the
ai-benchmark-equivalent suite (reference
README.md:248-251: VGG-16 b=20 224² inference / b=2 training, DeepLab b=2 512²
inference / b=1 384² training).

The reference measured TF-1 ai-benchmark graphs whose exact DeepLab variant
is not recorded in the repository, so the DeepLab here is architecture-
equivalent (parity unpinned); all weights are random-init.
"""
from __future__ import annotations

import os

import torch
from torch import nn
import torch.nn.functional as F

from vgpu.ops.bn import batched_step_counters, bn_act
from vgpu.ops.interp import resize_bilinear


class VGG16(nn.Module):
    cfg = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]

    def __init__(self, num_classes: int = 1000):
        super().__init__()
        layers: list[nn.Module] = []
        cin = 3
        for v in self.cfg:
            if v == "M":
                layers.append(nn.MaxPool2d(2, 2))
            else:
                layers += [nn.Conv2d(cin, v, 3, padding=1), nn.ReLU(inplace=True)]
                cin = v
        self.features = nn.Sequential(*layers)
        self.pool = nn.AdaptiveAvgPool2d((7, 7))
        self.classifier = nn.Sequential(
            nn.Linear(512 * 7 * 7, 4096), nn.ReLU(inplace=True),
            nn.Linear(4096, 4096), nn.ReLU(inplace=True),
            nn.Linear(4096, num_classes))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        train = self.training and torch.is_grad_enabled() and x.is_cuda
        if train:
            x = self._train_features(x)
        else:
            x = self.features(x)
        if x.shape[-2:] != (7, 7):
            x = self.pool(x)
        x = torch.flatten(x, 1)
        from vgpu.ops.conv import native_train_enabled
        if train and native_train_enabled():
            # batch ≤ 8: each FC layer + ReLU on the skinny kernels (vgpu.ops.linear)
            from vgpu.ops.linear import linear_act
            fc1, _, fc2, _, fc3 = self.classifier
            return linear_act(linear_act(linear_act(x.contiguous(), fc1, "relu"), fc2, "relu"), fc3)
        return self.classifier(x)

    def _train_features(self, x: torch.Tensor) -> torch.Tensor:
        """Training forward on the native kernels: each conv +
        ReLU pair with C % 64 == 0 is one MFMA conv with bias + ReLU in its
        epilogue and native data / weight gradients (vgpu.ops.conv.
        conv_bias_relu_train), max pools keep a one-byte argmax for a gather
        backward, and every stride-1 data-gradient filter is rebuilt by one
        batched launch per step.  Other shapes (the 3-channel first conv) run
        through the modules."""
        from vgpu.ops.conv import (DgradFilters, conv_bias_relu_pool_train, conv_bias_relu_train, maxpool_train,
                                   native_train_enabled)
        if native_train_enabled():
            if getattr(self, "_dgrad", None) is None:
                self._dgrad = DgradFilters([m for m in self.features if isinstance(m, nn.Conv2d)])
            self._dgrad.refresh()
        from vgpu.ops import conv as C
        C._RELU_LINK.clear()
        C._POOL_SRC.clear()
        x = x.contiguous(memory_format=torch.channels_last)
        mods = list(self.features)
        i = 0
        # what x is for the next conv: 0 anything, 1 the previous conv + ReLU's
        # output, 2 a fused conv + ReLU + pool block's output (each feeds only
        # the next conv here); the next conv's data gradient then does that
        # layer's ReLU (and pool) backward
        in_relu = 0
        while i < len(mods):
            m = mods[i]
            if isinstance(m, nn.Conv2d) and i + 1 < len(mods) and isinstance(mods[i + 1], nn.ReLU):
                if i + 2 < len(mods) and isinstance(mods[i + 2], nn.MaxPool2d):
                    # conv + ReLU + pool: the pool backward fused into the ReLU / bias gradient
                    # the last block writes NCHW: the classifier's flatten is then a view
                    x = conv_bias_relu_pool_train(x, m, mods[i + 2], in_relu=in_relu, out_nchw=i + 3 == len(mods))
                    i += 3
                    in_relu = 2
                    continue
                x = conv_bias_relu_train(x, m, in_relu=in_relu).contiguous(memory_format=torch.channels_last)
                i += 2
                in_relu = 1
                continue
            x = maxpool_train(x, m) if isinstance(m, nn.MaxPool2d) else m(x)
            i += 1
            in_relu = 0
        return x


class NativeVGG16Inference(nn.Module):
    """VGG-16 inference on the hand-written gfx950 kernels: every 3x3 convolution
    with C % 64 == 0 is the MFMA implicit-GEMM conv of native/kernels/conv_gemm.hip
    with bias + ReLU fused into its epilogue (one pass per layer instead of
    conv → bias → ReLU), max-pools are the NHWC pool kernel.  The 3-channel
    first layer stays on MIOpen.  Matches `VGG16.eval()` up to bf16 rounding
    (tests/test_gpu_conv.py)."""

    def __init__(self, m: VGG16):
        super().__init__()
        from vgpu.ops.conv import supported
        cl = torch.channels_last
        self.ops: list[tuple] = []
        with torch.no_grad():
            for mod in m.features:
                if isinstance(mod, nn.Conv2d):
                    w = mod.weight.detach().contiguous(memory_format=cl)
                    native = supported(mod.in_channels, mod.out_channels, mod.kernel_size[0])
                    b = mod.bias.detach().float().contiguous() if native else mod.bias.detach()
                    self.ops.append(("conv", w, b, native))
                elif isinstance(mod, nn.MaxPool2d):
                    self.ops.append(("pool", mod.kernel_size, mod.stride))
        self.pool = m.pool
        self.classifier = m.classifier

    @torch.no_grad()
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from vgpu.ops import conv as C
        x = x.contiguous(memory_format=torch.channels_last)
        for op in self.ops:
            if op[0] == "conv":
                _, w, b, native = op
                if native:
                    x = C.conv2d(x, w, b, padding=1, act="relu")
                else:
                    x = F.relu(F.conv2d(x, w, b, padding=1)).contiguous(memory_format=torch.channels_last)
            else:
                x = C.maxpool(x, op[1], op[2], 0)
        if x.shape[-2:] != (7, 7):
            x = self.pool(x)
        return self.classifier(torch.flatten(x, 1))


_ATROUS = os.environ.get("VGPU_ATROUS", "1") != "0"  # VGPU_ATROUS=0: dilated convs on MIOpen (A/B)
_ATROUS_INFER = os.environ.get("VGPU_ATROUS_INFER", "0") == "1"  # the BN-folded inference path too (A/B)


def _atrous_ok(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    """A dilated dense 3x3 conv (DeepLab's ASPP branches) that can run as a
    plain 3x3 on the space-to-batch sub-images (bf16 channels_last CUDA, C and
    Cout multiples of 64)."""
    d = conv.dilation[0]
    return (_ATROUS and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and conv.groups == 1 and d > 1
            and conv.dilation == (d, d) and conv.kernel_size == (3, 3) and conv.stride == (1, 1)
            and conv.padding == (d, d) and conv.in_channels % 64 == 0 and conv.out_channels % 64 == 0)


def _space_to_batch(x: torch.Tensor, d: int) -> torch.Tensor:
    """[N, C, H, W] -> [d·d·N, C, ⌈H/d⌉, ⌈W/d⌉]: sub-image (a, b) holds the
    pixels (a + d·i, b + d·j) (zero rows / columns past H, W), so a 3x3 conv
    with dilation d and padding d is a plain 3x3 / padding 1 conv on each
    sub-image (TF's atrous convolution).  Channels-last in and out, one copy:
    the permutation is taken on the NHWC storage itself."""
    n, c, h, w = x.shape
    hb, wb = -(-h // d), -(-w // d)
    if hb * d != h or wb * d != w:
        x = F.pad(x, (0, wb * d - w, 0, hb * d - h))
    xs = x.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1)  # NHWC view
    xs = xs.reshape(n, hb, d, wb, d, c).permute(2, 4, 0, 1, 3, 5).contiguous()
    return xs.view(d * d * n, hb, wb, c).permute(0, 3, 1, 2)


def _batch_to_space(y: torch.Tensor, d: int, n: int, h: int, w: int) -> torch.Tensor:
    c, hb, wb = y.shape[1:]
    yp = y.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1)  # NHWC view
    yp = yp.reshape(d, d, n, hb, wb, c).permute(2, 3, 0, 4, 1, 5).contiguous().view(n, hb * d, wb * d, c)
    if hb * d != h or wb * d != w:
        yp = yp[:, :h, :w, :].contiguous()
    return yp.permute(0, 3, 1, 2)


def _atrous_conv(x: torch.Tensor, conv: nn.Conv2d, w: torch.Tensor | None = None,
                 b: torch.Tensor | None = None, act: str = "none") -> torch.Tensor:
    """conv(x) for a dilated 3x3 (see _atrous_ok) on the native MFMA kernels
    via space-to-batch: training through vgpu.ops.conv's autograd conv (native
    data / weight gradients), or with a folded (w, b, act).  Training uses it
    (4.2: 367-373 -> 377 images/s, MIOpen's weight gradient alone was ~35 us a
    branch); the BN-folded inference keeps MIOpen's one forward kernel, which
    measured faster than the two copies + conv (4.1: 2 994 vs 2 925 images/s,
    scripts/pod_ab.sh)."""
    from vgpu.ops import conv as C
    d = conv.dilation[0]
    n, _, h, wd = x.shape
    xs = _space_to_batch(x, d)
    if w is None:
        y = C._ConvTrainFn.apply(xs, conv.weight, None, 1, 1)
    else:
        y = C.conv2d(xs, w, b, stride=1, padding=1, act=act)
    return _batch_to_space(y, d, n, h, wd)


class ConvBNAct(nn.Sequential):
    """conv → BatchNorm → (ReLU6); the BN + activation pair runs as one native
    training kernel pair (vgpu.ops.bn) on bf16 channels_last tensors.  On CUDA
    the conv is native too where a kernel exists: depthwise 3x3 (any stride /
    dilation, vgpu.ops.dwconv) and 1x1 / 3x3 with C, Cout % 64 == 0
    (vgpu.ops.conv.conv_train); the rest (the 3-channel stem, dilated ASPP
    convs, channel counts off the MFMA tiles) stay on the module."""

    def fuse(self) -> None:
        """Inference: fold the BatchNorm's running statistics into the conv
        (w' = w·s, b' = β - μ·s with s = γ / √(σ² + ε)), so the layer is one
        kernel with bias + activation in its epilogue.  Stale once trained again."""
        conv, bn = self[0], self[1]
        with torch.no_grad():
            s = bn.weight.float() / torch.sqrt(bn.running_var.float() + bn.eps)
            b = bn.bias.float() - bn.running_mean.float() * s
            if conv.bias is not None:
                b = b + conv.bias.float() * s
            w = (conv.weight.float() * s.view(-1, 1, 1, 1)).to(conv.weight.dtype)
        self._fused = (w.contiguous(memory_format=torch.channels_last), b.contiguous(),
                       w.float().reshape(w.shape[0], -1).t().contiguous() if conv.groups > 1 else None)

    def _forward_fused(self, x: torch.Tensor) -> torch.Tensor:
        from vgpu.ops import conv as C
        from vgpu.ops import dwconv
        conv = self[0]
        w, b, w9c = self._fused
        act = "relu6" if len(self) > 2 else "none"
        cl = x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous(memory_format=torch.channels_last)
        if cl and w9c is not None and dwconv.eligible(x, conv):
            return dwconv.dwconv3(x, w9c, conv.stride[0], conv.dilation[0], b, act)
        if cl and _ATROUS_INFER and _atrous_ok(x, conv):
            return _atrous_conv(x, conv, w, b, act)
        if (cl and conv.groups == 1 and conv.dilation == (1, 1) and conv.kernel_size[0] == conv.kernel_size[1]
                and conv.stride[0] == conv.stride[1] and conv.padding[0] == conv.padding[1]
                and C.supported(conv.in_channels, conv.out_channels, conv.kernel_size[0])
                and conv.kernel_size[0] in (1, 3)):
            return C.conv2d(x, w, b, stride=conv.stride[0], padding=conv.padding[0], act=act)
        y = F.conv2d(x, w, b.to(x.dtype), conv.stride, conv.padding, conv.dilation, conv.groups)
        return F.hardtanh_(y, 0.0, 6.0) if act == "relu6" else y

    def forward(self, x: torch.Tensor, res_out: bool = False, add: torch.Tensor | None = None):
        """act(bn(conv(x))) (+ add); res_out (1x1 / dense convs): also return x
        as an identity shortcut whose gradient the conv's data-gradient kernel
        sums in (vgpu.ops.conv.conv_train); add: a shortcut summed in the
        BatchNorm's own pass (vgpu.ops.bn.bn_act)."""
        conv = self[0]
        if not self.training and getattr(self, "_fused", None) is not None:
            y = self._forward_fused(x)
            y = y if add is None else y + add
            return (y, x) if res_out else y
        xs = x
        if x.is_cuda:
            from vgpu.ops import dwconv
            from vgpu.ops.conv import native_train_enabled
            if dwconv.eligible(x, conv):
                y = dwconv.dwconv_train(x, conv)
            elif native_train_enabled() and conv.bias is None and _atrous_ok(x, conv):
                y = _atrous_conv(x.contiguous(memory_format=torch.channels_last), conv)
            else:
                from vgpu.ops.conv import conv_train
                y = conv_train(x, conv, res_out=res_out)
                if res_out:
                    y, xs = y
        else:
            y = conv(x)
        y = bn_act(y, self[1], "relu6" if len(self) > 2 else "none", add=add)
        return (y, xs) if res_out else y


def _padc(c: int, pad: int) -> int:
    """Channel count stored for `c` real channels (a multiple of `pad`)."""
    return c if pad <= 1 else -(-c // pad) * pad


def _conv_bn(cin: int, cout: int, k: int, stride: int = 1, groups: int = 1, dilation: int = 1,
             act: bool = True, real: tuple[int, int] | None = None) -> nn.Sequential:
    """conv -> BN (-> ReLU6).  real = (input, output) channels that carry signal
    when cin / cout are padded: the padded weights, BN gammas and betas are zero,
    so padded channels stay exactly zero and receive exactly zero gradient
    (see MobileNetV2Backbone)."""
    pad = dilation * (k - 1) // 2
    mods: list[nn.Module] = [nn.Conv2d(cin, cout, k, stride, pad, dilation=dilation, groups=groups,
                                       bias=False), nn.BatchNorm2d(cout)]
    if act:
        mods.append(nn.ReLU6(inplace=True))
    m = ConvBNAct(*mods)
    if real is not None and real != (cin, cout):
        rin, rout = real
        with torch.no_grad():
            w = m[0].weight
            w[rout:] = 0
            if groups == 1:
                w[:, rin:] = 0
            m[1].weight[rout:] = 0
            m[1].bias[rout:] = 0
    return m


class InvertedResidual(nn.Module):
    def __init__(self, cin: int, cout: int, stride: int, expand: int, dilation: int = 1, pad: int = 1):
        super().__init__()
        hid = cin * expand
        self.use_res = stride == 1 and cin == cout
        pin, pout, phid = _padc(cin, pad), _padc(cout, pad), _padc(hid, pad)
        layers: list[nn.Module] = []
        if expand != 1:
            layers.append(_conv_bn(pin, phid, 1, real=(cin, hid)))
        layers += [_conv_bn(phid, phid, 3, stride, groups=phid, dilation=dilation, real=(hid, hid)),
                   _conv_bn(phid, pout, 1, act=False, real=(hid, cout))]
        self.body = nn.Sequential(*layers)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not self.use_res:
            return self.body(x)
        # the shortcut's gradient joins the first conv's data gradient in its
        # epilogue; the shortcut itself is added in the last BatchNorm's pass
        y, xs = self.body[0](x, res_out=True)
        for m in self.body[1:-1]:
            y = m(y)
        return self.body[-1](y, add=xs)


class MobileNetV2Backbone(nn.Module):
    """MobileNet-V2 (output stride 16).  pad > 1 stores every channel dimension
    rounded up to a multiple of `pad` (64: the native MFMA conv tiles; real
    widths 16, 24, 32, 96, 144 and 160 are not): the extra channels' weights,
    BN gammas and betas are zero, so they hold exact zeros in the forward, get
    exactly zero gradient in the backward (their BN gamma is 0; the weights
    reading them see zero inputs), and stay zero under SGD -- the network
    computes the same function with the same gradients on its real parameters
    as the unpadded one (tests/test_models_cpu.py), while every 1x1 conv runs
    on the native kernels instead of MIOpen."""
    # (expand, channels, repeats, stride) — output stride 16 with dilation in the last stages
    settings = [(1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1),
                (6, 160, 3, 1), (6, 320, 1, 1)]

    def __init__(self, pad: int = 1):
        super().__init__()
        self.pad = pad
        # the stem reads the image zero-padded to 64 channels too: a native conv
        # and weight gradient (~21x the MACs of 3 channels, still ~2 us) instead
        # of MIOpen's forward + weight gradient + helpers (~70 us a 4.2 step)
        layers: list[nn.Module] = [_conv_bn(_padc(3, pad), _padc(32, pad), 3, 2, real=(3, 32))]
        cin = 32
        dilation = 1
        for i, (t, c, n, s) in enumerate(self.settings):
            if i >= 5:
                dilation = 2
            for j in range(n):
                layers.append(InvertedResidual(cin, c, s if j == 0 else 1, t, dilation if j else 1, pad=pad))
                cin = c
        self.features = nn.Sequential(*layers)
        self.out_channels = _padc(cin, pad)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        cin = self.features[0][0].in_channels
        if x.shape[1] < cin:  # an RGB image into the channel-padded stem
            if x.is_cuda and x.dtype == torch.bfloat16:
                from vgpu.ops.conv import pad_channels
                x = pad_channels(x.contiguous(memory_format=torch.channels_last), cin)
            else:
                x = F.pad(x, (0, 0, 0, 0, 0, cin - x.shape[1]))
        return self.features(x)


class ASPP(nn.Module):
    def __init__(self, cin: int, cout: int = 256, rates=(6, 12, 18)):
        super().__init__()
        self.branches = nn.ModuleList([_conv_bn(cin, cout, 1)] +
                                      [_conv_bn(cin, cout, 3, dilation=r) for r in rates])
        self.image_pool = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Conv2d(cin, cout, 1, bias=False),
                                        nn.ReLU(inplace=True))
        self.project = _conv_bn(cout * (len(rates) + 2), cout, 1)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        h, w = x.shape[-2:]
        feats = [b(x) for b in self.branches]
        feats.append(resize_bilinear(self.image_pool(x), (h, w)))
        return self.project(torch.cat(feats, dim=1))


class DeepLabV3(nn.Module):
    """DeepLab-v3, MobileNet-V2 backbone + ASPP.  pad_channels: see
    MobileNetV2Backbone (64 by default: the same function, native convs)."""

    def __init__(self, num_classes: int = 21, pad_channels: int = 64):
        super().__init__()
        self.backbone = MobileNetV2Backbone(pad_channels)
        self.aspp = ASPP(self.backbone.out_channels)
        self.head = nn.Conv2d(256, num_classes, 1)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        h, w = x.shape[-2:]
        if self.training and torch.is_grad_enabled() and x.is_cuda:
            from vgpu.ops.conv import DgradFilters, native_train_enabled
            if native_train_enabled():
                # every 1x1 conv's transposed data-gradient filter in one launch per
                # step (a transpose copy per conv otherwise: 40 a step at 4.2)
                if getattr(self, "_dgrad", None) is None:
                    self._dgrad = DgradFilters([m for m in self.modules() if isinstance(m, nn.Conv2d)])
                self._dgrad.refresh()
        with batched_step_counters():
            y = self.head(self.aspp(self.backbone(x)))
        return resize_bilinear(y, (h, w))

    def load_unpadded(self, other: "DeepLabV3") -> None:
        """Copy an unpadded model's parameters and buffers into this (padded) one:
        each tensor into the leading slice of its padded counterpart; the padding
        stays zero (running variances of padded channels: 1)."""
        mine = dict(self.named_parameters()) | dict(self.named_buffers())
        with torch.no_grad():
            for name, t in list(other.named_parameters()) + list(other.named_buffers()):
                dst = mine[name]
                if dst.shape == t.shape:
                    dst.copy_(t)
                    continue
                if name.endswith("running_var"):
                    dst.fill_(1.0)
                else:
                    dst.zero_()
                dst[tuple(slice(0, n) for n in t.shape)].copy_(t)

    def fuse_for_inference(self) -> None:
        """Fold every conv → BatchNorm (→ ReLU6) into one conv with bias and
        activation in the kernel epilogue (ConvBNAct.fuse): 4.1 then runs
        one kernel per layer instead of a conv plus a BN-apply pass."""
        for m in self.modules():
            if isinstance(m, ConvBNAct):
                m.fuse()


class LSTMSentiment(nn.Module):
    """ai-benchmark "LSTM-Sentiment": 1024-token sequences of 300-d embeddings
    (reference README.md:252-253: inference b=100, training b=10)."""

    def __init__(self, emb: int = 300, hidden: int = 128, layers: int = 2, num_classes: int = 2):
        super().__init__()
        self.lstm = nn.LSTM(emb, hidden, num_layers=layers, batch_first=True)
        self.fc = nn.Linear(hidden, num_classes)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from vgpu.ops import lstm as fused
        if not self.training and fused.supported(self.lstm, x):
            return self.fc(fused.lstm_last_hidden(self.lstm, x))  # native recurrence kernel
        if self.training and fused.supported(self.lstm, x, training=True):
            return self.fc(fused.lstm_forward_train(self.lstm, x)[:, -1])  # native forward + backward kernels
        y, _ = self.lstm(x)
        return self.fc(y[:, -1])
