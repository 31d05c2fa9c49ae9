"""w13's input gradient from the transposed SwiGLU gradient only: if
dX = (dGU^T)^T W13 runs as fast as F.linear(dGU, W13^T), the SwiGLU
backward can skip writing the row-major dGU (940 MB per layer at
4x4096 tokens)."""
import torch

dev = torch.device("cuda", 0)
T, din, dout = 16384, 4096, 28672


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


dgu = torch.randn(T, dout, device=dev).bfloat16()
dgu_t = dgu.t().contiguous()
w = torch.randn(dout, din, device=dev).bfloat16()
wt = w.t().contiguous()
ref = torch.nn.functional.linear(dgu, wt).float()
for name, fn in [("linear(dGU, W^T)", lambda: torch.nn.functional.linear(dgu, wt)),
                 ("(dGU^T)^T (W^T)^T", lambda: torch.mm(dgu_t.t(), wt.t())),
                 ("(dGU^T)^T W", lambda: torch.mm(dgu_t.t(), w))]:
    t = timeit(fn)
    err = ((fn().float() - ref).abs().max() / ref.abs().max()).item()
    print(f"{name}: {t:.3f} ms ({2 * T * din * dout / t / 1e9:.0f} TF) err {err:.1e}", flush=True)
