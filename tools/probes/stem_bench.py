"""ResNet-50 stem conv at batch 256: the MFMA kernel (ops/stem.py) vs
MIOpen's bf16 channels-last conv, us per call (20 back-to-back calls)."""
import torch
import torch.nn as nn
import torch.nn.functional as F

from pytorch_operator_1_amd.ops.stem import _Stem

torch.backends.cudnn.benchmark = True
N = 256
x = torch.randn(N, 3, 224, 224, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
conv = nn.Conv2d(3, 64, 7, 2, 3, bias=False).cuda().to(memory_format=torch.channels_last)
wb = conv.weight.detach().bfloat16()


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


with torch.no_grad():
    t_k = timeit(lambda: _Stem.apply(x, conv.weight))
    t_m = timeit(lambda: F.conv2d(x, wb, stride=2, padding=3))
print(f"stem kernel {t_k:.1f} us | MIOpen conv {t_m:.1f} us")
