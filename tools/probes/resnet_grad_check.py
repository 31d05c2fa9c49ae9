"""ResNet-50 gradients at a given batch / image size: bf16 autocast (the
bench path, eager) vs an fp32 run of the same weights and data, per
parameter (relative error; 1.0 = the bf16 gradient is zero).  Also one
strided 1x1 conv's input gradient (MIOpen) vs fp32."""
import sys

import torch
import torch.nn.functional as F

from pytorch_operator_1_amd.models.resnet import resnet50, synthetic_images

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
IMG = int(sys.argv[2]) if len(sys.argv) > 2 else 224
torch.backends.cudnn.benchmark = True
dev = torch.device("cuda")
torch.manual_seed(0)
m = resnet50().to(dev, memory_format=torch.channels_last)
x, y = synthetic_images(B, dev, IMG, seed=0)


def grads(amp):
    m.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
        out = m(x)
    F.cross_entropy(out.float(), y).backward()
    torch.cuda.synchronize()
    return {n: p.grad.float().clone() for n, p in m.named_parameters()}


gb = grads(True)
gf = grads(False)
rows = []
for n in gf:
    ref = gf[n].norm().item()
    rows.append((((gb[n] - gf[n]).norm().item() / max(ref, 1e-30)), ref, gb[n].norm().item(), n))
rows.sort(reverse=True)
for r in rows[:16]:
    print(f"{r[3]:40s} rel {r[0]:.3e}  |fp32| {r[1]:.3e}  |bf16| {r[2]:.3e}")
# one strided 1x1 conv (layer2.0.downsample): MIOpen dgrad bf16 vs fp32
conv = m.layer2[0].downsample[0]
xi = torch.randn(B, 256, IMG // 4, IMG // 4, device=dev).contiguous(memory_format=torch.channels_last)
w = conv.weight.detach()
dy = torch.randn(B, 512, IMG // 8, IMG // 8, device=dev).contiguous(memory_format=torch.channels_last)
for dt in (torch.bfloat16, torch.float32):
    dx, dw, _ = torch.ops.aten.convolution_backward(dy.to(dt), xi.to(dt), w.to(dt), None, [2, 2], [0, 0], [1, 1],
                                                    False, [0, 0], 1, [True, True, False])
    torch.cuda.synchronize()
    print("strided 1x1", dt, "|dx|", dx.float().norm().item(), "|dw|", dw.float().norm().item())
