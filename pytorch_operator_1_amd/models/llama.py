"""Llama-3 decoder (BASELINE config 4: "Llama-3-8B DDP 8 replicas,
grad-bucket all-reduce stress, 288 GB HBM sizing").

The reference has no transformer workload (its only model is the MNIST
``Net`` of ``examples/mnist/mnist.py:12-28``); this is the framework's
large-model DDP config, built MI355X-first:

* bf16 parameters / activations; GEMMs on hipBLASLt through ``F.linear``
  with the projections fused to cut launches and re-reads: one QKV GEMM
  (``wqkv = [wq; wk; wv]``), one gate|up GEMM (``w13 = [w1; w3]``).
* Everything between GEMMs is one HIP kernel per boundary
  (:mod:`..ops.llm`): residual-add + RMSNorm (its backward also adds the
  residual-stream gradient), RoPE in place on the QKV output, SwiGLU, and
  the vocab-wide cross entropy on bf16 logits.
* Attention: ``F.scaled_dot_product_attention`` (causal, GQA) — the ROCm
  flash-attention path; q/k/v are strided views of the QKV output, so no
  transposes are materialised.
* Sizing: 8.03e9 params x (2 bf16 param + 2 bf16 grad + 12 fp32
  master/m/v) = 128 GB per GPU, leaving ~150 GB of the 288 GB HBM3E for
  activations (~4.4 MB/token without checkpointing), so a DDP replica
  holds 16-32k tokens per step with no sharding at all.

``impl="torch"`` is a plain PyTorch implementation of the same math used as
the numerics reference (and for CPU tests).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import torch
import torch.nn as nn
import torch.nn.functional as F

# impl="hip" attention: "hip" = csrc/kernels/attention.hip (head_dim 128,
# S % 128 == 0; other shapes fall back to SDPA), "sdpa" = ROCm SDPA.
ATTN_IMPL = os.environ.get("PTO_ATTN", "hip")


@dataclass
class LlamaConfig:
    dim: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: int = 8
    vocab_size: int = 128256
    ffn_dim: int = 14336
    rope_theta: float = 500000.0
    norm_eps: float = 1e-5
    max_seq_len: int = 8192
    rope_scaling: dict | None = field(default=None)
    tie_embeddings: bool = False

    @property
    def head_dim(self) -> int:
        return self.dim // self.n_heads

    def num_params(self) -> int:
        hd = self.head_dim
        attn = self.dim * (self.n_heads + 2 * self.n_kv_heads) * hd + self.n_heads * hd * self.dim
        mlp = 3 * self.dim * self.ffn_dim
        per_layer = attn + mlp + 2 * self.dim
        emb = self.vocab_size * self.dim * (1 if self.tie_embeddings else 2)
        return self.n_layers * per_layer + emb + self.dim

    def train_flops_per_token(self, seq_len: int) -> float:
        """6N (dense) + causal attention 6 * L * S * dim (fwd+bwd)."""
        n_dense = self.num_params() - self.vocab_size * self.dim  # embedding lookup is not a GEMM
        return 6.0 * n_dense + 6.0 * self.n_layers * seq_len * self.dim


CONFIGS = {
    "llama3-8b": LlamaConfig(),
    "llama3-1b": LlamaConfig(dim=2048, n_layers=16, n_heads=32, n_kv_heads=8, ffn_dim=8192),
    "llama3-tiny": LlamaConfig(dim=256, n_layers=2, n_heads=8, n_kv_heads=2, vocab_size=1024, ffn_dim=512,
                               max_seq_len=256),
}


def _rotate_half(x):
    a, b = x.chunk(2, dim=-1)
    return torch.cat((-b, a), dim=-1)


class LlamaBlock(nn.Module):
    def __init__(self, cfg: LlamaConfig, device=None, dtype=None):
        super().__init__()
        kw = dict(device=device, dtype=dtype)
        hd = cfg.head_dim
        self.cfg = cfg
        self.attn_norm = nn.Parameter(torch.ones(cfg.dim, **kw))
        self.wqkv = nn.Linear(cfg.dim, (cfg.n_heads + 2 * cfg.n_kv_heads) * hd, bias=False, **kw)
        self.wo = nn.Linear(cfg.n_heads * hd, cfg.dim, bias=False, **kw)
        self.ffn_norm = nn.Parameter(torch.ones(cfg.dim, **kw))
        self.w13 = nn.Linear(cfg.dim, 2 * cfg.ffn_dim, bias=False, **kw)
        self.w2 = nn.Linear(cfg.ffn_dim, cfg.dim, bias=False, **kw)

    # -- attention core shared by both impls (qkv already rotated) --
    def _attend(self, qkv, B, S):
        c = self.cfg
        hd = c.head_dim
        v4 = qkv.view(B, S, c.n_heads + 2 * c.n_kv_heads, hd)
        q = v4[:, :, :c.n_heads].transpose(1, 2)
        k = v4[:, :, c.n_heads:c.n_heads + c.n_kv_heads].transpose(1, 2)
        v = v4[:, :, c.n_heads + c.n_kv_heads:].transpose(1, 2)
        # GQA without materialising repeated K/V (measured 0.70 vs 0.87 ms fwd
        # at 2x4096 tokens, plus no expand copies: profiles/llama8b_ops_r1.json)
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=c.n_kv_heads != c.n_heads)
        return o.transpose(1, 2).reshape(B * S, c.n_heads * hd)

    def forward_hip(self, h, delta, rope, B, S):
        from ..ops import llm

        c = self.cfg
        if delta is None:
            y = llm.rmsnorm(h, self.attn_norm, c.norm_eps)
        else:
            h, y = llm.add_rmsnorm(h, delta, self.attn_norm, c.norm_eps)
        qkv = _lin(y, self.wqkv)
        qkv = llm.rope_(qkv, rope[0], rope[1], S, c.n_heads + c.n_kv_heads, c.head_dim)
        if ATTN_IMPL == "hip" and llm.flash_attention_supported(S, c.n_heads, c.n_kv_heads, c.head_dim):
            ctx = llm.flash_attention(qkv, B, S, c.n_heads, c.n_kv_heads)  # [B*S, H*128], no transposes
        else:
            ctx = self._attend(qkv, B, S)
        attn = _lin(ctx, self.wo)
        h, y = llm.add_rmsnorm(h, attn, self.ffn_norm, c.norm_eps)
        # the SwiGLU backward hands w13's weight gradient its output
        # gradient already transposed (ops/llm.py TStash)
        st = llm.TStash() if getattr(self.w13, "dw_kcontig", False) and os.environ.get("PTO_SWIGLU_T", "1") == "1" \
            else None
        mlp = _lin(llm.swiglu(_lin(y, self.w13, st), st), self.w2)
        return h, mlp

    def forward_torch(self, h, delta, rope, B, S):
        c = self.cfg
        if delta is not None:
            h = h + delta
        y = _rmsnorm_ref(h, self.attn_norm, c.norm_eps)
        qkv = F.linear(y, self.wqkv.weight)
        nr = (c.n_heads + c.n_kv_heads) * c.head_dim
        rot = qkv[:, :nr].reshape(B, S, -1, c.head_dim).float()
        cos = torch.cat([rope[0], rope[0]], -1)[None, :, None, :]
        sin = torch.cat([rope[1], rope[1]], -1)[None, :, None, :]
        rot = (rot * cos + _rotate_half(rot) * sin).to(qkv.dtype).reshape(B * S, nr)
        qkv = torch.cat([rot, qkv[:, nr:]], dim=1)
        attn = F.linear(self._attend(qkv, B, S), self.wo.weight)
        h = h + attn
        y = _rmsnorm_ref(h, self.ffn_norm, c.norm_eps)
        g, u = F.linear(y, self.w13.weight).chunk(2, dim=-1)
        mlp = F.linear(F.silu(g) * u, self.w2.weight)
        return h, mlp


def _lin(x, mod: nn.Linear, tstash=None):
    """Bias-free linear; with a transposed weight copy attached
    (:meth:`Llama.enable_transposed_dgrad`) the input gradient uses it."""
    wt = getattr(mod, "weight_t", None)
    if wt is None:
        return F.linear(x, mod.weight)
    from ..ops import llm

    return llm.linear_tw(x, mod.weight, wt, getattr(mod, "dw_kcontig", False), tstash)


def _rmsnorm_ref(x, w, eps):
    xf = x.float()
    n = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return w * n.to(x.dtype)


class Llama(nn.Module):
    def __init__(self, cfg: LlamaConfig | str = "llama3-8b", impl: str = "hip", device=None,
                 dtype=torch.bfloat16, checkpoint: str = "none", init_std: float = 0.02):
        super().__init__()
        if isinstance(cfg, str):
            cfg = CONFIGS[cfg]
        if impl not in ("hip", "torch"):
            raise ValueError(f"impl must be hip|torch, got {impl}")
        if checkpoint not in ("none", "full"):
            raise ValueError("checkpoint must be none|full")
        self.cfg, self.impl, self.checkpoint = cfg, impl, checkpoint
        kw = dict(device=device, dtype=dtype)
        self.tok_emb = nn.Embedding(cfg.vocab_size, cfg.dim, **kw)
        self.layers = nn.ModuleList(LlamaBlock(cfg, **kw) for _ in range(cfg.n_layers))
        self.norm = nn.Parameter(torch.ones(cfg.dim, **kw))
        self.lm_head = None if cfg.tie_embeddings else nn.Linear(cfg.dim, cfg.vocab_size, bias=False, **kw)
        self._rope = {}
        self.reset_parameters(init_std)

    @torch.no_grad()
    def reset_parameters(self, std: float = 0.02):
        out_std = std / math.sqrt(2 * self.cfg.n_layers)  # scaled residual-branch outputs
        for name, p in self.named_parameters():
            if p.dim() == 1:
                p.fill_(1.0)
            elif name.endswith("wo.weight") or name.endswith("w2.weight"):
                p.normal_(0.0, out_std)
            else:
                p.normal_(0.0, std)

    def rope(self, S: int, device):
        key = (S, str(device))
        if key not in self._rope:
            from ..ops.llm import rope_tables

            self._rope[key] = rope_tables(S, self.cfg.head_dim, self.cfg.rope_theta, device, self.cfg.rope_scaling)
        return self._rope[key]

    def linear_modules(self):
        mods = [m for blk in self.layers for m in (blk.wqkv, blk.wo, blk.w13, blk.w2)]
        return mods + ([self.lm_head] if self.lm_head is not None else [])

    def _mark_kcontig_dw(self):
        """Weight-gradient GEMMs that run faster from transposed activations
        (measured per shape, tools/dw_layout_bench.py): wo and w13."""
        for blk in self.layers:
            blk.wo.dw_kcontig = True
            blk.w13.dw_kcontig = True

    @torch.no_grad()
    def enable_transposed_dgrad(self):
        """Keep ``W^T`` next to every linear weight (bf16, +1x weight memory:
        16 GB for Llama-3-8B) so each dgrad GEMM reads K-contiguous operands.
        The copies must be refreshed after every weight update
        (:meth:`refresh_transposed`)."""
        for m in self.linear_modules():
            if getattr(m, "weight_t", None) is None:
                w = m.weight
                m.weight_t = torch.empty(w.shape[1], w.shape[0], device=w.device, dtype=w.dtype)
        self._mark_kcontig_dw()
        self.refresh_transposed()

    @torch.no_grad()
    def refresh_transposed(self):
        from ..ops import llm

        for m in self.linear_modules():
            wt = getattr(m, "weight_t", None)
            if wt is not None:
                llm.transpose_into(m.weight, wt)

    def _head_weight(self):
        return self.tok_emb.weight if self.lm_head is None else self.lm_head.weight

    def forward(self, tokens: torch.Tensor, labels: torch.Tensor | None = None):
        """``tokens`` [B, S] int64 -> mean CE loss if ``labels`` given, else logits."""
        B, S = tokens.shape
        rope = self.rope(S, tokens.device)
        h = self.tok_emb(tokens).reshape(B * S, self.cfg.dim)
        delta = None
        for blk in self.layers:
            fn = blk.forward_hip if self.impl == "hip" else blk.forward_torch
            if self.checkpoint == "full" and self.training and torch.is_grad_enabled():
                from torch.utils.checkpoint import checkpoint

                h, delta = checkpoint(fn, h, delta, rope, B, S, use_reentrant=False)
            else:
                h, delta = fn(h, delta, rope, B, S)
        if self.impl == "hip":
            from ..ops import llm

            _, y = llm.add_rmsnorm(h, delta, self.norm, self.cfg.norm_eps)
            logits = F.linear(y, self._head_weight()) if self.lm_head is None else _lin(y, self.lm_head)
            if labels is None:
                return logits.view(B, S, -1)
            return llm.cross_entropy(logits, labels.reshape(-1))
        h = h + delta
        y = _rmsnorm_ref(h, self.norm, self.cfg.norm_eps)
        logits = F.linear(y, self._head_weight())
        if labels is None:
            return logits.view(B, S, -1)
        return F.cross_entropy(logits.float(), labels.reshape(-1))


def synthetic_tokens(batch: int, seq_len: int, vocab: int, device, seed: int = 0):
    """Random token ids + next-token labels (no dataset access: synthetic)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    t = torch.randint(0, vocab, (batch, seq_len + 1), generator=g)
    return t[:, :-1].contiguous().to(device), t[:, 1:].contiguous().to(device)
