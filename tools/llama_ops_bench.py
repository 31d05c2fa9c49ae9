#!/usr/bin/env python3
"""Per-op timing of one Llama-3-8B layer at the bench shape (tokens=B*S):
GEMMs (hipBLASLt), attention variants, and the HIP kernels between them,
forward and backward, plus the optimizer and the LM head + CE.  Device time
from HIP events, median of N.  Prints a table and writes JSON.

Usage: python tools/llama_ops_bench.py [--batch 2] [--seq 4096] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch.nn.functional as F


def timed(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--seq", type=int, default=4096)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    from pytorch_operator_1_amd.models.llama import CONFIGS
    from pytorch_operator_1_amd.ops import llm

    c = CONFIGS["llama3-8b"]
    dev = "cuda"
    B, S, D, H, KV, hd, Fd, V = args.batch, args.seq, c.dim, c.n_heads, c.n_kv_heads, c.head_dim, c.ffn_dim, c.vocab_size
    M = B * S
    bf = dict(device=dev, dtype=torch.bfloat16)
    res = {}

    def gemm(name, m, n, k):
        x = torch.randn(m, k, **bf)
        w = torch.randn(n, k, **bf) * 0.02
        dy = torch.randn(m, n, **bf)
        t = timed(lambda: F.linear(x, w))
        tb = timed(lambda: (dy @ w, dy.t() @ x))
        fl = 2.0 * m * n * k
        res[name] = {"fwd_ms": t, "bwd_ms": tb, "fwd_tflops": fl / t / 1e9, "bwd_tflops": 2 * fl / tb / 1e9}

    gemm("wqkv", M, (H + 2 * KV) * hd, D)
    gemm("wo", M, D, H * hd)
    gemm("w13", M, 2 * Fd, D)
    gemm("w2", M, D, Fd)
    gemm("lm_head", M, V, D)

    # attention variants
    qkv = torch.randn(M, (H + 2 * KV) * hd, **bf)
    v4 = qkv.view(B, S, H + 2 * KV, hd)
    q = v4[:, :, :H].transpose(1, 2)
    k = v4[:, :, H:H + KV].transpose(1, 2)
    v = v4[:, :, H + KV:].transpose(1, 2)
    attn_fl = 4.0 * B * H * S * S * hd / 2  # causal

    def expand(t):
        return t[:, :, None].expand(B, KV, H // KV, S, hd).reshape(B, H, S, hd)

    for name, fn in {
        "sdpa_expand": lambda: F.scaled_dot_product_attention(q, expand(k), expand(v), is_causal=True),
        "sdpa_gqa": lambda: F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True),
    }.items():
        try:
            t = timed(fn)
            qq = q.detach().clone().requires_grad_()
            kk = k.detach().clone().requires_grad_()
            vv = v.detach().clone().requires_grad_()
            if name == "sdpa_expand":
                o = F.scaled_dot_product_attention(qq, expand(kk), expand(vv), is_causal=True)
            else:
                o = F.scaled_dot_product_attention(qq, kk, vv, is_causal=True, enable_gqa=True)
            go = torch.randn_like(o)
            tb = timed(lambda: torch.autograd.grad(o, (qq, kk, vv), go, retain_graph=True))
            res[name] = {"fwd_ms": t, "bwd_ms": tb, "fwd_tflops": attn_fl / t / 1e9, "bwd_tflops": 2.5 * attn_fl / tb / 1e9}
        except Exception as e:  # noqa: BLE001
            res[name] = {"error": repr(e)[:200]}
    try:  # hand-written gfx950 flash attention straight from the QKV layout
        fa_in = qkv.clone()
        t = timed(lambda: llm.flash_attention(fa_in, B, S, H, KV))
        a = fa_in.clone().requires_grad_()
        o = llm.flash_attention(a, B, S, H, KV)
        go = torch.randn_like(o)
        tb = timed(lambda: torch.autograd.grad(o, a, go, retain_graph=True))
        res["flash_hip"] = {"fwd_ms": t, "bwd_ms": tb, "fwd_tflops": attn_fl / t / 1e9, "bwd_tflops": 2.5 * attn_fl / tb / 1e9}
    except Exception as e:  # noqa: BLE001
        res["flash_hip"] = {"error": repr(e)[:200]}
    try:
        from torch.nn.attention import SDPBackend, sdpa_kernel

        for be in ("FLASH_ATTENTION", "EFFICIENT_ATTENTION", "MATH"):
            try:
                with sdpa_kernel(getattr(SDPBackend, be)):
                    t = timed(lambda: F.scaled_dot_product_attention(q, expand(k), expand(v), is_causal=True), iters=3)
                res[f"sdpa_backend_{be}"] = {"fwd_ms": t}
            except Exception as e:  # noqa: BLE001
                res[f"sdpa_backend_{be}"] = {"error": repr(e)[:160]}
    except ImportError:
        pass

    # HIP kernels between GEMMs
    x = torch.randn(M, D, **bf)
    r = torch.randn(M, D, **bf)
    w = torch.ones(D, **bf)
    res["add_rmsnorm_fwd"] = {"fwd_ms": timed(lambda: llm.add_rmsnorm(x, r, w))}
    xr = x.clone().requires_grad_()
    rr = r.clone().requires_grad_()
    h, y = llm.add_rmsnorm(xr, rr, w.clone().requires_grad_())
    gy = torch.randn_like(y)
    res["add_rmsnorm_bwd"] = {"bwd_ms": timed(lambda: torch.autograd.grad((h, y), (xr, rr), (gy, gy), retain_graph=True))}
    gu = torch.randn(M, 2 * Fd, **bf)
    res["swiglu_fwd"] = {"fwd_ms": timed(lambda: llm.swiglu(gu))}
    res["rope_fwd"] = {"fwd_ms": timed(lambda: llm.rope_(qkv, *llm.rope_tables(S, hd, 5e5, dev), S, H + KV, hd))}
    logits = torch.randn(M, V, **bf)
    labels = torch.randint(0, V, (M,), device=dev)
    res["ce_fwd"] = {"fwd_ms": timed(lambda: llm.cross_entropy(logits, labels))}
    # bytes-based bandwidth for the memory-bound ops
    res["add_rmsnorm_fwd"]["GBps"] = 4 * M * D * 2 / res["add_rmsnorm_fwd"]["fwd_ms"] / 1e6
    res["swiglu_fwd"]["GBps"] = 3 * M * Fd * 2 / res["swiglu_fwd"]["fwd_ms"] / 1e6
    res["ce_fwd"]["GBps"] = M * V * 2 / res["ce_fwd"]["fwd_ms"] / 1e6

    # optimizer over 8B bf16 params is measured in the model bench; here one 1 GB tensor
    from pytorch_operator_1_amd.ops.optim import FusedAdamW

    p = torch.randn(V * D, **bf).requires_grad_()
    p.grad = torch.randn_like(p)
    opt = FusedAdamW([p])
    opt.step()
    t = timed(lambda: opt.step(), iters=5)
    res["adamw_1GB_bf16"] = {"ms": t, "GBps": p.numel() * (2 + 2 + 12 + 2 + 12) / t / 1e6}

    for k_, v_ in res.items():
        print(f"{k_:28s} " + "  ".join(f"{a}={b:.3f}" if isinstance(b, float) else f"{a}={b}" for a, b in v_.items()))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
