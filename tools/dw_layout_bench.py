"""Llama-3-8B weight-gradient GEMM layouts (4x4096 tokens): dW = dY^T X as
autograd computes it (both operands MN-contiguous) vs from transposed
activations (both K-contiguous) plus the cost of the two transposes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_operator_1_amd.ops import llm  # noqa: E402

dev = torch.device("cuda", 0)
T = 16384


def timeit(fn, n=10):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


for name, din, dout in [("wqkv", 4096, 6144), ("wo", 4096, 4096), ("w13", 4096, 28672), ("w2", 14336, 4096)]:
    x = torch.randn(T, din, device=dev).bfloat16()
    dy = torch.randn(T, dout, device=dev).bfloat16()
    xt = torch.empty(din, T, device=dev, dtype=torch.bfloat16)
    dyt = torch.empty(dout, T, device=dev, dtype=torch.bfloat16)
    fl = 2 * T * din * dout
    t_std = timeit(lambda: dy.t().mm(x))
    llm.transpose_into(x, xt)
    llm.transpose_into(dy, dyt)
    t_k = timeit(lambda: dyt.mm(xt.t()))
    t_tr = timeit(lambda: (llm.transpose_into(x, xt), llm.transpose_into(dy, dyt)))
    err = ((dyt.mm(xt.t()).float() - dy.t().mm(x).float()).abs().max() / dy.t().mm(x).float().abs().max()).item()
    print(f"{name}: dY^T X {t_std:.3f} ms ({fl / t_std / 1e9:.0f} TF) | K-contig {t_k:.3f} ms ({fl / t_k / 1e9:.0f} TF)"
          f" + transposes {t_tr:.3f} ms | rel err {err:.1e}", flush=True)
