"""Llama-3-8B weight gradients whose output tiles do not fill the chip in
whole waves (4x4096 tokens, 256x256 hipBLASLt tiles on 256 CUs):
wqkv [6144 x 4096] = 384 tiles (1.5 waves), w2 [4096 x 14336] = 896 tiles
(3.5 waves).  Variants: split-K batched GEMM with fp32 partials + one
summing pass to bf16, and the dW GEMM on a side stream next to the dgrad
GEMM of the same layer."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorch_operator_1_amd.ops import llm  # noqa: E402

dev = torch.device("cuda", 0)
T = 16384


def timeit(fn, n=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


side = torch.cuda.Stream()
for name, din, dout in [("wqkv", 4096, 6144), ("wo", 4096, 4096), ("w13", 4096, 28672), ("w2", 14336, 4096)]:
    x = torch.randn(T, din, device=dev).bfloat16()
    dy = torch.randn(T, dout, device=dev).bfloat16()
    wt = torch.randn(din, dout, device=dev).bfloat16()
    xt = torch.empty(din, T, device=dev, dtype=torch.bfloat16)
    dyt = torch.empty(dout, T, device=dev, dtype=torch.bfloat16)
    llm.transpose_into(x, xt)
    llm.transpose_into(dy, dyt)
    fl = 2 * T * din * dout
    ref = dy.t().mm(x).float()
    out = torch.empty(dout, din, device=dev, dtype=torch.bfloat16)
    line = [f"{name}: dY^T X {timeit(lambda: dy.t().mm(x)):.3f}",
            f"K-contig {timeit(lambda: dyt.mm(xt.t())):.3f}"]
    for S in (2, 4):
        a = dy.view(S, T // S, dout).transpose(1, 2)
        b = x.view(S, T // S, din)
        ak = dyt.view(dout, S, T // S).permute(1, 0, 2)
        bk = xt.view(din, S, T // S).permute(1, 2, 0)
        part = torch.empty(S, dout, din, device=dev, dtype=torch.float32)

        def sk(a=a, b=b, part=part):
            torch.bmm(a, b, out_dtype=torch.float32, out=part)
            out.copy_(part.sum(0))

        def skk(a=ak, b=bk, part=part):
            torch.bmm(a, b, out_dtype=torch.float32, out=part)
            out.copy_(part.sum(0))

        t1 = timeit(sk)
        err1 = ((out.float() - ref).abs().max() / ref.abs().max()).item()
        t2 = timeit(skk)
        err2 = ((out.float() - ref).abs().max() / ref.abs().max()).item()
        tb = timeit(lambda: torch.bmm(a, b, out_dtype=torch.float32, out=part))
        line.append(f"splitK{S} {t1:.3f} (gemm {tb:.3f}, err {err1:.0e}) K-contig splitK{S} {t2:.3f} (err {err2:.0e})")
    t_dg = timeit(lambda: torch.nn.functional.linear(dy, wt))
    t_seq = timeit(lambda: (torch.nn.functional.linear(dy, wt), dy.t().mm(x)))

    def conc():
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            dy.t().mm(x)
        torch.nn.functional.linear(dy, wt)
        torch.cuda.current_stream().wait_stream(side)

    t_conc = timeit(conc)
    line.append(f"dgrad {t_dg:.3f} | dgrad+dW serial {t_seq:.3f} side-stream {t_conc:.3f}")
    print(" | ".join(line) + f"  ({fl / 1e12:.2f} TFLOP each)", flush=True)
