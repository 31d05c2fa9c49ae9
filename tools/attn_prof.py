#!/usr/bin/env python3
"""Run the flash attention fwd + bwd at the Llama-3-8B bench shape a few
times (for rocprofv3 kernel traces / PMC counters)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_operator_1_amd.ops import llm  # noqa: E402

B, S, H, KV = int(os.environ.get("B", 4)), 4096, 32, 8
qkv = torch.randn(B * S, (H + 2 * KV) * 128, device="cuda", dtype=torch.bfloat16).requires_grad_()
for _ in range(int(os.environ.get("ITERS", 3))):
    o = llm.flash_attention(qkv, B, S, H, KV)
    o.backward(torch.ones_like(o))
torch.cuda.synchronize()
print("ok")
