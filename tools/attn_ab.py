#!/usr/bin/env python3
"""Time the flash attention forward / backward at the Llama-3-8B bench
shape (B x 4096 tokens, 32 query / 8 KV heads, head dim 128) and report
TF/s (causal FLOPs: 4 B H S^2 D / 2 forward, 2.5x that backward).

Kernel variants are chosen by env vars read once per process
(PTO_ATTN_DKDV_PC, PTO_ATTN_PC_KVWAIT), so A/B runs are separate processes:
    for v in 0 2 4; do PTO_ATTN_DKDV=$v python tools/attn_ab.py; done
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_operator_1_amd.ops import llm  # noqa: E402


def main():
    B, S, H, KV = int(os.environ.get("B", 4)), int(os.environ.get("S", 4096)), 32, 8
    iters = int(os.environ.get("ITERS", 20))
    torch.manual_seed(0)
    qkv = torch.randn(B * S, (H + 2 * KV) * 128, device="cuda", dtype=torch.bfloat16)
    a = qkv.clone().requires_grad_()
    o = llm.flash_attention(a, B, S, H, KV)
    go = torch.randn_like(o)

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters

    tf = timed(lambda: llm.flash_attention(qkv, B, S, H, KV))
    tb = timed(lambda: torch.autograd.grad(o, a, go, retain_graph=True))
    fl = 4.0 * B * H * S * S * 128 / 2
    g = torch.autograd.grad(o, a, go, retain_graph=True)[0]
    print(json.dumps({"dkdv_pc": os.environ.get("PTO_ATTN_DKDV_PC", "default"),
                      "pc_kvwait": os.environ.get("PTO_ATTN_PC_KVWAIT", "default"), "B": B, "S": S,
                      "fwd_ms": round(tf, 4), "bwd_ms": round(tb, 4), "fwd_tflops": round(fl / tf / 1e9, 1),
                      "bwd_tflops": round(2.5 * fl / tb / 1e9, 1),
                      "grad_checksum": float(g.float().abs().sum().item())}), flush=True)


if __name__ == "__main__":
    main()
