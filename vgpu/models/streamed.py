"""Llama inference with layer weights paged between pinned host memory and a
bounded HBM working set (virtual device memory, BASELINE.json config 5).

Each decoder block's parameters are packed into one flat chunk registered
with the HostPager; the forward pass prefetches `lookahead` blocks ahead on the
pager stream while the current block computes (double/triple buffering), so
the run is bounded by host→HBM bandwidth, not by copy latency.  Blocks that
fit the budget stay resident across tokens (LRU), so a budget of B bytes
streams only (model − B) per token.
"""
from __future__ import annotations

import torch
from torch import nn
from torch.func import functional_call

from vgpu.ops.pager import HostPager

from .llama import Llama, LlamaConfig


class FlatLayout:
    def __init__(self, module: nn.Module):
        self.entries = []
        off = 0
        self.dtype = None
        for name, p in module.named_parameters():
            self.dtype = self.dtype or p.dtype
            n = p.numel()
            self.entries.append((name, tuple(p.shape), off, n))
            off += n
        self.numel = off

    def pack(self, module: nn.Module) -> torch.Tensor:
        flat = torch.empty(self.numel, dtype=self.dtype)
        for (name, _, off, n), (_, p) in zip(self.entries, module.named_parameters()):
            flat[off:off + n].copy_(p.detach().reshape(-1).to("cpu"))
        return flat

    def views(self, flat: torch.Tensor) -> dict[str, torch.Tensor]:
        return {name: flat[off:off + n].view(shape) for name, shape, off, n in self.entries}


class StreamedLlama:
    def __init__(self, model: Llama, budget_bytes: int, device="cuda", lookahead: int = 2):
        self.model = model
        self.device = torch.device(device)
        self.lookahead = lookahead
        self.pager = HostPager(budget_bytes, self.device)
        # small parts stay resident
        self.embed = model.embed.to(self.device)
        self.norm = model.norm.to(self.device)
        self.head = model.head.to(self.device)
        self.layout = FlatLayout(model.layers[0])
        self.n = len(model.layers)
        self.template = model.layers[0]
        for i, blk in enumerate(model.layers):
            self.pager.register(f"L{i}", self.layout.pack(blk))
        # free the original host copies of the layers (the pager owns them now)
        model.layers = nn.ModuleList()
        self.template = self.template.to(self.device)

    @classmethod
    def random_init(cls, cfg, budget_bytes: int, device="cuda", lookahead: int = 2,
                    dtype=torch.bfloat16, std: float = 0.02) -> "StreamedLlama":
        """Random-init weights generated per block on the GPU and parked in pinned
        host memory (an 8B model never needs to fit in HBM at once)."""
        from .llama import Block
        self = cls.__new__(cls)
        self.device = torch.device(device)
        self.lookahead = lookahead
        self.pager = HostPager(budget_bytes, self.device)
        with torch.device("meta"):
            shell = Llama(LlamaConfig(**{**cfg.__dict__, "layers": 1}))
        self.model = shell
        self.model.cfg = cfg
        self.embed = nn.Embedding(cfg.vocab, cfg.dim, device=self.device, dtype=dtype)
        nn.init.normal_(self.embed.weight, std=std)
        self.norm = shell.norm.to_empty(device=self.device).to(dtype)
        nn.init.ones_(self.norm.weight)
        self.head = nn.Linear(cfg.dim, cfg.vocab, bias=False, device=self.device, dtype=dtype)
        nn.init.normal_(self.head.weight, std=std)
        with torch.device("meta"):
            tmpl = Block(cfg).to(dtype)
        self.layout = FlatLayout(tmpl)
        self.n = cfg.layers
        g = torch.Generator(device=self.device).manual_seed(0)
        for i in range(cfg.layers):
            flat = torch.randn(self.layout.numel, generator=g, device=self.device, dtype=dtype) * std
            for name, shape, off, n in self.layout.entries:
                if name.endswith("norm1.weight") or name.endswith("norm2.weight"):
                    flat[off:off + n] = 1
            self.pager.register(f"L{i}", flat)
            del flat
        self.template = tmpl.to_empty(device=self.device)
        return self

    def n_resident(self) -> int:
        """Layers kept permanently in HBM.  A decoder scans its layers cyclically,
        which is LRU's worst case (every layer misses once the model exceeds the
        budget), so the pager pins a prefix of the layers and streams only the
        rest through a ring of `lookahead + 1` slots."""
        if getattr(self, "policy", "pin-prefix") == "lru":
            return 0
        slots = self.pager.budget // max(self.layer_bytes(), 1)
        if slots >= self.n:
            return self.n
        return max(0, min(self.n, slots - (self.lookahead + 1)))

    @torch.inference_mode()
    def forward(self, tokens: torch.Tensor, kv_caches=None, pos: int = 0) -> torch.Tensor:
        cos, sin = self.model.rope(self.device)
        x = self.embed(tokens)
        n_res = self.n_resident()
        # the ring fills while the resident prefix computes
        first = n_res if n_res < self.n else 0
        self.pager.prefetch([f"L{j}" for j in range(first, min(first + self.lookahead, self.n))])
        for i in range(self.n):
            name = f"L{i}"
            self.pager.pin(name)
            flat = self.pager.get(name)
            if i + 1 >= n_res:
                lo = max(i + 1, n_res)
                self.pager.prefetch([f"L{j}" for j in range(lo, min(i + 1 + self.lookahead, self.n))])
            params = self.layout.views(flat)
            kv = kv_caches[i] if kv_caches is not None else None
            x = functional_call(self.template, params, (x, cos, sin, kv, pos))
            if i >= n_res:
                self.pager.unpin(name)
        return self.head(self.norm(x[:, -1:]))

    __call__ = forward

    def layer_bytes(self) -> int:
        return self.pager.nbytes("L0")
