"""Llama-3-8B RMSNorm backward (16384 x 4096 bf16, residual gradient on):
time per call of pto_rmsnorm_bwd (row kernel + column sums) and its
effective bandwidth (reads dy, h, dres; writes dx)."""
import torch

from pytorch_operator_1_amd.ops import _lib

L = _lib.lib()
M, D = 16384, 4096
dev = torch.device("cuda", 0)
dy, h, dres = (torch.randn(M, D, device=dev).bfloat16() for _ in range(3))
w = torch.randn(D, device=dev).bfloat16()
rstd = torch.rand(M, device=dev) + 0.5
dx = torch.empty_like(dy)
dw = torch.empty_like(w)
part = torch.empty(L.pto_rmsnorm_bwd_groups(M), D, device=dev)
s = _lib.stream_ptr()


def call():
    L.pto_rmsnorm_bwd(dy.data_ptr(), h.data_ptr(), w.data_ptr(), rstd.data_ptr(), dres.data_ptr(), dx.data_ptr(),
                      dw.data_ptr(), part.data_ptr(), M, D, s)


for _ in range(3):
    call()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50):
    call()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / 50 * 1e3
print(f"rmsnorm_bwd {us:.1f} us ({4 * M * D * 2 / us / 1e6:.2f} TB/s) checksum {dx.float().abs().sum().item():.6e}",
      flush=True)
