"""Fused BN(+ReLU) HIP kernels vs MIOpen batch norm + ReLU on ResNet-50's
channels-last bf16 shapes (batch 256): forward and forward+backward time
and effective bandwidth."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_operator_1_amd.ops.bn import BatchNormAct  # noqa: E402

dev = torch.device("cuda", 0)


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3  # us


for C, HW in [(64, 112), (64, 56), (256, 56), (128, 28), (512, 28), (1024, 14), (2048, 7)]:
    x = torch.randn(256, C, HW, HW, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    dy = torch.randn_like(x)
    m = BatchNormAct(C).to(dev)
    nbytes = x.numel() * 2
    res = {}
    for mode in ("fused", "miopen"):
        os.environ["PTO_FUSED_BN"] = "1" if mode == "fused" else "0"

        def fwd():
            return m(x, relu=True)

        def fwdbwd():
            y = m(x, relu=True)
            y.backward(dy)

        with torch.no_grad():
            tf = timeit(lambda: m(x.detach(), relu=True))
        tb = timeit(fwdbwd)
        res[mode] = (tf, tb)
    f, mi = res["fused"], res["miopen"]
    print(f"C={C:5d} HW={HW:3d} ({nbytes / 1e6:6.0f} MB): fwd fused {f[0]:7.1f} us ({3 * nbytes / f[0] / 1e6:5.2f} TB/s eff) "
          f"miopen {mi[0]:7.1f} us | fwd+bwd fused {f[1]:7.1f} us miopen {mi[1]:7.1f} us", flush=True)
