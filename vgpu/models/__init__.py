"""Workload registry: the ai-benchmark-equivalent suite the reference's
published numbers are quoted on (reference README.md:244-253),
plus Llama-3 for the virtual-device-memory scenario.

Each entry: (builder, input factory, batch, resolution) for inference and
training exactly as listed in the reference README.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable

import torch
from torch import nn

from .llama import Llama, LlamaConfig
from .resnet import resnet_v2_50, resnet_v2_152
from .vision import VGG16, DeepLabV3, LSTMSentiment


@dataclass(frozen=True)
class Workload:
    test_id: str          # ai-benchmark test id (README.md:244-253)
    name: str
    builder: Callable[[], nn.Module]
    batch: int
    shape: tuple          # per-sample input shape
    train: bool
    kind: str = "image"   # image | sequence
    baseline_exclusive: float = 0.0   # images/s, BASELINE.md (2xV100)
    baseline_vgpu: float = 0.0
    baseline_vmem: float = 0.0

    def make_input(self, device, dtype=torch.bfloat16, gen: torch.Generator | None = None):
        x = torch.randn((self.batch, *self.shape), device=device, dtype=dtype, generator=gen)
        if self.kind == "image":
            x = x.contiguous(memory_format=torch.channels_last)
        return x


WORKLOADS: dict[str, Workload] = {w.test_id: w for w in [
    Workload("1.1", "resnet_v2_50", resnet_v2_50, 50, (3, 346, 346), False,
             baseline_exclusive=135.86, baseline_vgpu=141.2, baseline_vmem=207.9),
    Workload("1.2", "resnet_v2_50", resnet_v2_50, 20, (3, 346, 346), True,
             baseline_exclusive=45.24, baseline_vgpu=43.68, baseline_vmem=79.84),
    Workload("2.1", "resnet_v2_152", resnet_v2_152, 10, (3, 256, 256), False,
             baseline_exclusive=110.0, baseline_vgpu=102.0, baseline_vmem=211.3),
    Workload("2.2", "resnet_v2_152", resnet_v2_152, 10, (3, 256, 256), True,
             baseline_exclusive=32.67, baseline_vgpu=30.2, baseline_vmem=45.14),
    Workload("3.1", "vgg16", VGG16, 20, (3, 224, 224), False,
             baseline_exclusive=137.9, baseline_vgpu=134.2, baseline_vmem=179.77),
    Workload("3.2", "vgg16", VGG16, 2, (3, 224, 224), True,
             baseline_exclusive=8.62, baseline_vgpu=8.62, baseline_vmem=14.87),
    Workload("4.1", "deeplab", DeepLabV3, 2, (3, 512, 512), False,
             baseline_exclusive=8.97, baseline_vgpu=8.92, baseline_vmem=11.1),
    Workload("4.2", "deeplab", DeepLabV3, 1, (3, 384, 384), True,
             baseline_exclusive=4.15, baseline_vgpu=4.09, baseline_vmem=7.69),
    Workload("5.1", "lstm", LSTMSentiment, 100, (1024, 300), False, kind="sequence",
             baseline_exclusive=22.78, baseline_vgpu=22.32, baseline_vmem=23.02),
    Workload("5.2", "lstm", LSTMSentiment, 10, (1024, 300), True, kind="sequence",
             baseline_exclusive=4.66, baseline_vgpu=3.96, baseline_vmem=6.95),
]}

__all__ = ["WORKLOADS", "Workload", "Llama", "LlamaConfig", "resnet_v2_50", "resnet_v2_152",
           "VGG16", "DeepLabV3", "LSTMSentiment"]
