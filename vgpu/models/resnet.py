"""ResNet-V2 (pre-activation) — the ai-benchmark ResNet-V2-50 / ResNet-V2-152
workloads the reference publishes numbers for (BASELINE.md rows 1.x / 2.x;
reference README.md:244-247: ResNet-V2-50 b=50 346² inference, b=20 346²
training; ResNet-V2-152 b=10 256²).

Random init, NCHW module layout run in channels_last memory format so MIOpen
picks its NHWC (CK) kernels on gfx950.  `fuse_for_inference()` folds every
BatchNorm that directly follows a convolution into that convolution's weights,
leaving only the block-entry pre-activation BNs (which sit after a residual
add and cannot be folded).
"""
from __future__ import annotations

import torch
from torch import nn
import torch.nn.functional as F

from vgpu.ops import bnconv
from vgpu.ops.bn import batched_step_counters, bn_act, bn_act_res
from vgpu.ops.conv import DgradFilters, conv_train, maxpool_train
from vgpu.ops.conv import native_train_enabled as _conv_train_native


class PreActBottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, width: int, stride: int):
        super().__init__()
        cout = width * self.expansion
        self.bn_in = nn.BatchNorm2d(cin)
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, cout, 1, bias=False)
        self.shortcut = None
        if stride != 1 or cin != cout:
            self.shortcut = nn.Conv2d(cin, cout, 1, stride=stride, bias=False)
        self.fused = False

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.shortcut is None and not self.fused and torch.is_grad_enabled():
            # identity shortcut: its gradient is summed into bn_in's backward
            pre, x = bn_act_res(x, self.bn_in)
        else:
            pre = bn_act(x, self.bn_in)
        if self.fused:
            sc = self.shortcut(pre) if self.shortcut is not None else x
            y = F.relu(self.conv1(pre))
            y = F.relu(self.conv2(y))
            return self.conv3(y) + sc
        # training / unfused: MFMA convs (residual add in conv3's epilogue) and
        # native BN+ReLU on bf16 channels_last CUDA tensors, PyTorch elsewhere
        sc = conv_train(pre, self.shortcut) if self.shortcut is not None else x
        y = bn_act(conv_train(pre, self.conv1), self.bn1)
        y = bn_act(conv_train(y, self.conv2), self.bn2)
        return conv_train(y, self.conv3, residual=sc)

    def forward_fused(self, x: torch.Tensor, st: torch.Tensor | None):
        """Training step with the BatchNorm statistics carried by the convs
        (vgpu.ops.bnconv): `st` are x's (Σ, Σ²) pairs from the previous block's
        conv3 epilogue (None: reduced here); returns (out, out's pairs)."""
        if self.shortcut is None:
            h1, st1, x = bnconv.bn_conv(x, self.bn_in, self.conv1, stats_in=st, res_out=True)
            sc = x
        else:
            h1, st1, sc = bnconv.bn_conv(x, self.bn_in, self.conv1, stats_in=st, shortcut=self.shortcut)
        h2, st2 = bnconv.bn_conv(h1, self.bn1, self.conv2, stats_in=st1)
        return bnconv.bn_conv(h2, self.bn2, self.conv3, residual=sc, stats_in=st2)

    def fused_eligible(self, x: torch.Tensor) -> bool:
        # the block's inner tensors share x's dtype / device / layout; every
        # ResNet-V2 conv has C, Cout % 64 == 0 (bn_conv falls back per shape)
        return not self.fused and torch.is_grad_enabled() and bnconv.eligible(x, self.bn_in, self.conv1)


def _fold_bn(conv: nn.Conv2d, bn: nn.BatchNorm2d) -> nn.Conv2d:
    w = conv.weight.detach()
    scale = bn.weight.detach() / torch.sqrt(bn.running_var + bn.eps)
    new = nn.Conv2d(conv.in_channels, conv.out_channels, conv.kernel_size, conv.stride,
                    conv.padding, conv.dilation, conv.groups, bias=True)
    new.weight.data = (w * scale.reshape(-1, 1, 1, 1)).to(w.dtype)
    b = conv.bias.detach() if conv.bias is not None else torch.zeros_like(bn.running_mean)
    new.bias.data = ((b - bn.running_mean) * scale + bn.bias.detach()).to(w.dtype)
    return new.to(w.device)


class ResNetV2(nn.Module):
    def __init__(self, layers: list[int], num_classes: int = 1000):
        super().__init__()
        self.stem = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.pool = nn.MaxPool2d(3, stride=2, padding=1)
        blocks = []
        cin = 64
        for i, (n, width) in enumerate(zip(layers, (64, 128, 256, 512))):
            for j in range(n):
                stride = 2 if (j == 0 and i > 0) else 1
                blocks.append(PreActBottleneck(cin, width, stride))
                cin = width * PreActBottleneck.expansion
        self.blocks = nn.Sequential(*blocks)
        self.bn_out = nn.BatchNorm2d(cin)
        self.fc = nn.Linear(cin, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.training and torch.is_grad_enabled() and x.is_cuda and _conv_train_native():
            # every stride-1 conv's data-gradient filter in one launch (vgpu.ops.conv.DgradFilters)
            if getattr(self, "_dgrad", None) is None:
                self._dgrad = DgradFilters([m for m in self.modules() if isinstance(m, nn.Conv2d)])
            self._dgrad.refresh()
        with batched_step_counters():
            x = self.stem(x)
            x = maxpool_train(x, self.pool) if self.training and torch.is_grad_enabled() else self.pool(x)
            if self.training and all(b.fused_eligible(x) for b in self.blocks[:1]):
                st = None
                for b in self.blocks:
                    x, st = b.forward_fused(x, st)
            else:
                x = self.blocks(x)
            x = bn_act(x, self.bn_out)
        x = torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
        return self.fc(x)

    @torch.no_grad()
    def fuse_for_inference(self) -> "ResNetV2":
        for b in self.blocks:
            b.conv1 = _fold_bn(b.conv1, b.bn1)
            b.conv2 = _fold_bn(b.conv2, b.bn2)
            b.bn1 = nn.Identity()
            b.bn2 = nn.Identity()
            b.fused = True
        return self


class FusedResNetV2Inference(nn.Module):
    """Inference runner for a ResNetV2 with every BN folded.

    conv="native" (default): every convolution after the stem is the MFMA
    implicit-GEMM kernel of native/kernels/conv_gemm.hip with its neighbours
    fused in — the block-entry BN+ReLU as the prologue of conv1 and of the
    projection shortcut, folded-BN bias + ReLU as the epilogue of conv1/conv2,
    the residual add as the epilogue of conv3 — so a bottleneck is 3 (or 4)
    kernels and the pre-activation tensor is never materialised.  The stem
    7x7/s2 stem runs as space-to-depth + a 4x4 narrow-C MFMA conv; its
    max-pool and the final BN+ReLU+global-mean are hand-written kernels too.

    conv="miopen": MIOpen convolutions + the fused NHWC epilogues of
    vgpu.ops.fused (3 activation passes per bottleneck instead of 7).

    Both are numerically equivalent to `ResNetV2.eval()` up to bf16 rounding
    (tests/test_gpu_fused.py, tests/test_gpu_conv.py).
    """

    def __init__(self, m: ResNetV2, conv: str = "native"):
        super().__init__()
        if conv not in ("native", "miopen"):
            raise ValueError(conv)
        self.conv = conv
        # conv2+conv3 fusion (VGPU_FUSE_TAIL=0 disables, for A/B)
        import os
        self.fuse_tail = os.environ.get("VGPU_FUSE_TAIL", "1") != "0"
        # ... and the next identity block's conv1 into that tail (VGPU_FUSE_NEXT=0 disables)
        self.fuse_next = self.fuse_tail and os.environ.get("VGPU_FUSE_NEXT", "1") != "0"
        from vgpu.ops.fused import bn_scale_shift
        m = m.eval()
        dt = m.stem.weight.dtype
        cl = torch.channels_last

        def fold(conv: nn.Conv2d, bn: nn.BatchNorm2d):
            scale = bn.weight.float() / torch.sqrt(bn.running_var.float() + bn.eps)
            w = (conv.weight.float() * scale.reshape(-1, 1, 1, 1)).to(dt).contiguous(memory_format=cl)
            b = (bn.bias.float() - bn.running_mean.float() * scale).contiguous()
            return w, b

        with torch.no_grad():
            self.stem_w = m.stem.weight.detach().contiguous(memory_format=cl)
            if conv == "native":
                from vgpu.ops.conv import stem_weight_s2d
                self.stem_w_s2d = stem_weight_s2d(self.stem_w)
            self.blocks = []
            for blk in m.blocks:
                w1, b1 = fold(blk.conv1, blk.bn1)
                w2, b2 = fold(blk.conv2, blk.bn2)
                self.blocks.append({
                    "in": bn_scale_shift(blk.bn_in),
                    "w1": w1, "b1": b1, "w2": w2, "b2": b2,
                    "stride": blk.conv2.stride[0],
                    "w3": blk.conv3.weight.detach().contiguous(memory_format=cl),
                    "sc": None if blk.shortcut is None else
                    (blk.shortcut.weight.detach().contiguous(memory_format=cl), blk.shortcut.stride[0]),
                })
            self.out_ss = bn_scale_shift(m.bn_out)
            self.fc = m.fc

    @torch.no_grad()
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.conv == "native":
            return self._forward_native(x)
        return self._forward_miopen(x)

    def _forward_native(self, x: torch.Tensor) -> torch.Tensor:
        from vgpu.ops import conv as C
        x = x.contiguous(memory_format=torch.channels_last)
        x = C.stem_pool(x, self.stem_w_s2d)  # stem conv + max pool, one kernel
        x = self._blocks_native(x, 0, len(self.blocks))
        return self.fc(C.scale_shift_relu_mean(x, *self.out_ss))

    def _blocks_native(self, x: torch.Tensor, first: int, last: int) -> torch.Tensor:
        """Blocks [first, last); `last` must start a stage (or be the end) so no
        fused next-block conv1 output crosses the boundary."""
        from vgpu.ops import conv as C
        h_next = None
        for i in range(first, last):
            b = self.blocks[i]
            pro = b["in"]
            if b["sc"] is None:
                sc = x
            else:
                sc = C.conv2d(x, b["sc"][0], stride=b["sc"][1], pro=pro)
            h = h_next if h_next is not None else C.conv2d(x, b["w1"], b["b1"], act="relu", pro=pro)
            h_next = None
            nb = self.blocks[i + 1] if i + 1 < last else None
            if (self.fuse_next and nb is not None and nb["sc"] is None
                    and C.conv23_supported(h.shape[1])):
                # conv2 + conv3 + residual + the next block's BN+ReLU+conv1 (stages 1-2)
                x, h_next = C.conv231(h, b["w2"], b["b2"], b["w3"], sc, nb["w1"], nb["b1"], nb["in"],
                                      stride=b["stride"])
            elif self.fuse_tail and C.conv23_supported(h.shape[1]):
                # conv2 + conv3 + residual in one kernel (stages 1-2)
                x = C.conv23(h, b["w2"], b["b2"], b["w3"], sc, stride=b["stride"])
            else:
                h = C.conv2d(h, b["w2"], b["b2"], stride=b["stride"], padding=1, act="relu")
                x = C.conv2d(h, b["w3"], residual=sc)
        return x

    def _forward_miopen(self, x: torch.Tensor) -> torch.Tensor:
        from vgpu.ops.fused import add_scale_shift_act, bias_act_, scale_shift_act
        x = F.max_pool2d(F.conv2d(x, self.stem_w, stride=2, padding=3), 3, 2, 1)
        x = x.contiguous(memory_format=torch.channels_last)
        pre = scale_shift_act(x, *self.blocks[0]["in"])
        n = len(self.blocks)
        for i, b in enumerate(self.blocks):
            if b["sc"] is None:
                sc = x
            else:
                sc = F.conv2d(pre, b["sc"][0], stride=b["sc"][1])
            h = bias_act_(F.conv2d(pre, b["w1"]), b["b1"])
            h = bias_act_(F.conv2d(h, b["w2"], stride=b["stride"], padding=1), b["b2"])
            h = F.conv2d(h, b["w3"])
            nss = self.blocks[i + 1]["in"] if i + 1 < n else self.out_ss
            x, pre = add_scale_shift_act(h, sc, *nss)
        pooled = pre.mean(dim=(2, 3))
        return self.fc(pooled)


def resnet_v2_50(num_classes: int = 1000) -> ResNetV2:
    return ResNetV2([3, 4, 6, 3], num_classes)


def resnet_v2_152(num_classes: int = 1000) -> ResNetV2:
    return ResNetV2([3, 8, 36, 3], num_classes)
