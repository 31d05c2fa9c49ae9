"""ResNetTrainer: eager vs eager vs whole-step graph, per-tensor relative
distance of the final state (|a - b| / |b - init|)."""
import sys

import torch

from pytorch_operator_1_amd.train.bench_models import ResNetTrainer


def run(graph, steps, lr):
    tr = ResNetTrainer(torch.device("cuda"), batch_size=8, image_size=64, lr=lr, seed=3, graph=graph)
    init = {k: v.detach().float().clone() for k, v in tr.model.state_dict().items()}
    losses = []
    for _ in range(steps):
        tr.step()
        losses.append(tr.last_loss())
    torch.cuda.synchronize()
    return init, {k: v.detach().float().clone() for k, v in tr.model.state_dict().items()}, losses


steps, lr = int(sys.argv[1]), float(sys.argv[2])
i0, a, la = run(False, steps, lr)
_, b, lb = run(False, steps, lr)
_, c, lc = run(True, steps, lr)
print("losses eager", [round(x, 5) for x in la])
print("losses eager2", [round(x, 5) for x in lb])
print("losses graph", [round(x, 5) for x in lc])
worst = []
for k in a:
    if not a[k].is_floating_point():
        print(k, a[k].item() if a[k].numel() == 1 else "", c[k].item() if c[k].numel() == 1 else "")
        continue
    mv = (a[k] - i0[k]).norm().item() + 1e-12
    worst.append(((c[k] - a[k]).norm().item() / mv, (b[k] - a[k]).norm().item() / mv, k))
worst.sort(reverse=True)
for w in worst[:15]:
    print(f"{w[2]:40s} graph-eager {w[0]:.3e}  eager-eager {w[1]:.3e}")
