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

# the transposed product dW^T = X^T dY [din, dout] (what an optimizer that
# reads the gradient transposed could take): same FLOPs, other tile shapes
print("--- dW^T forms", flush=True)
for name, din, dout in [("wqkv", 4096, 6144), ("wo", 4096, 4096), ("w13", 4096, 28672), ("w2", 14336, 4096)]:
    x = torch.randn(T, din, device=dev).bfloat16()
    dy = torch.randn(T, dout, device=dev).bfloat16()
    xt = torch.empty(din, T, device=dev, dtype=torch.bfloat16)
    dyt = torch.empty(dout, T, device=dev, dtype=torch.bfloat16)
    llm.transpose_into(x, xt)
    llm.transpose_into(dy, dyt)
    w = torch.randn(dout, din, device=dev).bfloat16()
    fl = 2 * T * din * dout
    t_a = timeit(lambda: x.t().mm(dy))
    t_b = timeit(lambda: xt.mm(dyt.t()))
    t_f = timeit(lambda: torch.nn.functional.linear(x, w))
    print(f"{name}: X^T dY {t_a:.3f} ms ({fl / t_a / 1e9:.0f} TF) | K-contig X^T dY {t_b:.3f} ms "
          f"({fl / t_b / 1e9:.0f} TF) | forward x W^T {t_f:.3f} ms ({fl / t_f / 1e9:.0f} TF)", flush=True)

# input gradient dX = dY W: from W itself (B operand N-contiguous) vs from the
# W^T copy the step keeps (K-contiguous, what F.linear(dY, W^T) runs)
print("--- dgrad forms", flush=True)
for name, din, dout in [("wqkv", 4096, 6144), ("wo", 4096, 4096), ("w13", 4096, 28672), ("w2", 14336, 4096)]:
    dy = torch.randn(T, dout, device=dev).bfloat16()
    w = torch.randn(dout, din, device=dev).bfloat16()
    wt = w.t().contiguous()
    fl = 2 * T * din * dout
    t_w = timeit(lambda: dy.mm(w))
    t_wt = timeit(lambda: torch.nn.functional.linear(dy, wt))
    print(f"{name}: dY W {t_w:.3f} ms ({fl / t_w / 1e9:.0f} TF) | dY (W^T)^T {t_wt:.3f} ms ({fl / t_wt / 1e9:.0f} TF)",
          flush=True)
