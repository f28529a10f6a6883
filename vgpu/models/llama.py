"""Llama-3 decoder (random init) for the virtual-device-memory workload
(BASELINE.json config 5: "one pod requests gpumem=400000M on a 288 GB MI355X,
Llama-3-8B random-init inference via host-swap paging").

Standard architecture: RMSNorm, RoPE (theta 500k), grouped-query attention
through F.scaled_dot_product_attention (flash/CK path on ROCm), SwiGLU MLP,
untied embeddings.  `LlamaConfig.llama3_8b()` is the 8B shape; tests use
`LlamaConfig.tiny()`.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
from torch import nn
import torch.nn.functional as F


@dataclass
class LlamaConfig:
    vocab: int = 128256
    dim: int = 4096
    layers: int = 32
    heads: int = 32
    kv_heads: int = 8
    ffn: int = 14336
    rope_theta: float = 500000.0
    max_seq: int = 8192
    eps: float = 1e-5

    @staticmethod
    def llama3_8b() -> "LlamaConfig":
        return LlamaConfig()

    @staticmethod
    def tiny() -> "LlamaConfig":
        return LlamaConfig(vocab=512, dim=128, layers=2, heads=4, kv_heads=2, ffn=256, max_seq=256)


class RMSNorm(nn.Module):
    def __init__(self, dim: int, eps: float):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(dim))
        self.eps = eps

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        xf = x.float()
        y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.eps)
        return (y * self.weight.float()).to(x.dtype)


def rope_tables(cfg: LlamaConfig, device=None) -> tuple[torch.Tensor, torch.Tensor]:
    hd = cfg.dim // cfg.heads
    inv = 1.0 / (cfg.rope_theta ** (torch.arange(0, hd, 2, device=device).float() / hd))
    t = torch.arange(cfg.max_seq, device=device).float()
    f = torch.outer(t, inv)
    return f.cos(), f.sin()


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    # x: [B, H, S, D]; cos/sin: [S, D/2]
    x1, x2 = x.float().chunk(2, dim=-1)
    c, s = cos[None, None], sin[None, None]
    return torch.cat([x1 * c - x2 * s, x1 * s + x2 * c], dim=-1).to(x.dtype)


class Attention(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.h, self.kvh, self.hd = cfg.heads, cfg.kv_heads, cfg.dim // cfg.heads
        self.wqkv = nn.Linear(cfg.dim, (cfg.heads + 2 * cfg.kv_heads) * self.hd, bias=False)
        self.wo = nn.Linear(cfg.dim, cfg.dim, bias=False)

    def forward(self, x, cos, sin, kv_cache=None, pos: int = 0):
        B, S, _ = x.shape
        qkv = self.wqkv(x)
        q, k, v = qkv.split([self.h * self.hd, self.kvh * self.hd, self.kvh * self.hd], dim=-1)
        q = q.view(B, S, self.h, self.hd).transpose(1, 2)
        k = k.view(B, S, self.kvh, self.hd).transpose(1, 2)
        v = v.view(B, S, self.kvh, self.hd).transpose(1, 2)
        q = apply_rope(q, cos[pos:pos + S], sin[pos:pos + S])
        k = apply_rope(k, cos[pos:pos + S], sin[pos:pos + S])
        if kv_cache is not None:
            kc, vc = kv_cache
            kc[:, :, pos:pos + S] = k
            vc[:, :, pos:pos + S] = v
            k, v = kc[:, :, :pos + S], vc[:, :, :pos + S]
        rep = self.h // self.kvh
        if rep > 1:
            k = k.repeat_interleave(rep, dim=1)
            v = v.repeat_interleave(rep, dim=1)
        o = F.scaled_dot_product_attention(q, k, v, is_causal=(S > 1))
        return self.wo(o.transpose(1, 2).reshape(B, S, -1))


class Block(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.norm1 = RMSNorm(cfg.dim, cfg.eps)
        self.attn = Attention(cfg)
        self.norm2 = RMSNorm(cfg.dim, cfg.eps)
        self.w13 = nn.Linear(cfg.dim, 2 * cfg.ffn, bias=False)
        self.w2 = nn.Linear(cfg.ffn, cfg.dim, bias=False)

    def forward(self, x, cos, sin, kv_cache=None, pos: int = 0):
        x = x + self.attn(self.norm1(x), cos, sin, kv_cache, pos)
        g, u = self.w13(self.norm2(x)).chunk(2, dim=-1)
        return x + self.w2(F.silu(g) * u)


class Llama(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        self.embed = nn.Embedding(cfg.vocab, cfg.dim)
        self.layers = nn.ModuleList([Block(cfg) for _ in range(cfg.layers)])
        self.norm = RMSNorm(cfg.dim, cfg.eps)
        self.head = nn.Linear(cfg.dim, cfg.vocab, bias=False)
        self._rope = None

    def rope(self, device):
        if self._rope is None or self._rope[0].device != device:
            self._rope = rope_tables(self.cfg, device)
        return self._rope

    def forward(self, tokens: torch.Tensor, kv_caches=None, pos: int = 0) -> torch.Tensor:
        cos, sin = self.rope(tokens.device)
        x = self.embed(tokens)
        for i, layer in enumerate(self.layers):
            x = layer(x, cos, sin, kv_caches[i] if kv_caches is not None else None, pos)
        return self.head(self.norm(x[:, -1:]))

    @torch.no_grad()
    def decode_static(self, tokens: torch.Tensor, kv_caches, pos: torch.Tensor) -> torch.Tensor:
        """One decode step with every shape fixed (graph-capturable): `pos` is
        a 1-element device tensor, the cache is written with index_copy_ and
        attention runs over the whole cache with positions > pos masked."""
        cos, sin = self.rope(tokens.device)
        c, s_ = cos.index_select(0, pos), sin.index_select(0, pos)
        x = self.embed(tokens)
        B = x.shape[0]
        ctx = kv_caches[0][0].shape[2]
        mask = (torch.arange(ctx, device=tokens.device) <= pos)[None, None, None, :]
        for i, layer in enumerate(self.layers):
            a = layer.attn
            h = layer.norm1(x)
            q, k, v = a.wqkv(h).split([a.h * a.hd, a.kvh * a.hd, a.kvh * a.hd], dim=-1)
            q = apply_rope(q.view(B, 1, a.h, a.hd).transpose(1, 2), c, s_)
            k = apply_rope(k.view(B, 1, a.kvh, a.hd).transpose(1, 2), c, s_)
            v = v.view(B, 1, a.kvh, a.hd).transpose(1, 2)
            kc, vc = kv_caches[i]
            kc.index_copy_(2, pos, k)
            vc.index_copy_(2, pos, v)
            rep = a.h // a.kvh
            kk = kc.repeat_interleave(rep, dim=1) if rep > 1 else kc
            vv = vc.repeat_interleave(rep, dim=1) if rep > 1 else vc
            o = F.scaled_dot_product_attention(q, kk, vv, attn_mask=mask)
            x = x + a.wo(o.transpose(1, 2).reshape(B, 1, -1))
            g, u = layer.w13(layer.norm2(x)).chunk(2, dim=-1)
            x = x + layer.w2(F.silu(g) * u)
        return self.head(self.norm(x))

    def new_kv_cache(self, batch: int, seq: int, dtype=torch.bfloat16, device=None):
        hd = self.cfg.dim // self.cfg.heads
        shape = (batch, self.cfg.kv_heads, seq, hd)
        return [(torch.empty(shape, dtype=dtype, device=device),
                 torch.empty(shape, dtype=dtype, device=device)) for _ in range(self.cfg.layers)]
