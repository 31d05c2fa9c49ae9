"""Llama-3-8B projection GEMMs (4x4096 tokens) under hipBLASLt vs rocBLAS
(torch.backends.cuda.preferred_blas_library): forward, dgrad from W^T and
the weight gradients in the layouts the step uses."""
import torch
import torch.nn.functional as F

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


for name, din, dout in [("wqkv", 4096, 6144), ("wo", 4096, 4096), ("w13", 4096, 28672), ("w2", 14336, 4096)]:
    x = torch.randn(T, din, device=dev).bfloat16()
    dy = torch.randn(T, dout, device=dev).bfloat16()
    w = torch.randn(dout, din, device=dev).bfloat16()
    wt = w.t().contiguous()
    xt, dyt = x.t().contiguous(), dy.t().contiguous()
    forms = {"fwd": lambda: F.linear(x, w), "dgrad": lambda: F.linear(dy, wt),
             "dW dY^T X": lambda: dy.t().mm(x), "dW K-contig": lambda: dyt.mm(xt.t())}
    line = []
    for fname, fn in forms.items():
        r = []
        for lib in ("cublaslt", "cublas"):
            torch.backends.cuda.preferred_blas_library(lib)
            r.append(timeit(fn))
        line.append(f"{fname} lt {r[0]:.3f} / rocblas {r[1]:.3f}")
    torch.backends.cuda.preferred_blas_library("cublaslt")
    print(f"{name}: " + " | ".join(line), flush=True)
