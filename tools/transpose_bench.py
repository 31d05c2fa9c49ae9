"""Bandwidth of the bf16 transpose kernel on the Llama-3-8B weight shapes."""
import torch

from pytorch_operator_1_amd.ops import llm

dev = torch.device("cuda", 0)
for r, c in [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (128256, 4096)]:
    x = torch.randn(r, c, device=dev).bfloat16()
    y = torch.empty(c, r, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        llm.transpose_into(x, y)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        llm.transpose_into(x, y)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 20
    assert torch.equal(y, x.t())
    print(f"transpose {r}x{c}: {ms * 1e3:.1f} us, {2 * r * c * 2 / ms / 1e9:.2f} TB/s", flush=True)
