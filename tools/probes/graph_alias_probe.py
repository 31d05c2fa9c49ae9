"""Whole-step HIP graph of ResNetTrainer at lr = 0: every replay must
compute the same gradients (the state does not change), so any buffer the
captured step reads but does not (re)write inside the graph shows up as a
drift between replays.  Also replays after eager NaN-filled allocations (a
graph node pointing at memory freed during capture would pick them up).
Usage: graph_alias_probe.py [batch] [image]"""
import sys

import torch

from pytorch_operator_1_amd.train.bench_models import ResNetTrainer

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
IMG = int(sys.argv[2]) if len(sys.argv) > 2 else 64
tr = ResNetTrainer(torch.device("cuda"), batch_size=B, image_size=IMG, lr=0.0, seed=3, graph=True)
named = list(tr.model.named_parameters())
eager = {}
_release = tr.bucketer.release


def snap_release():  # the eager steps' gradients, before they are dropped: the reference
    eager.clear()
    eager.update({n: p.grad.float().clone() for n, p in named if p.grad is not None})
    _release()


tr.bucketer.release = snap_release
tr.run(2)
tr.bucketer.release = _release
ref = dict(eager)
ref_loss = tr.last_loss()
tr.step()  # capture + first replay


def check(tag):
    torch.cuda.synchronize()
    bad = []
    for n, p in named:
        g = p.grad.float()
        if not torch.isfinite(g).all() or not torch.isfinite(p).all():
            bad.append(f"{n}:nonfinite")
            continue
        d = ((g - ref[n]).norm() / ref[n].norm().clamp_min(1e-20)).item()
        if d > 2e-2:
            bad.append(f"{n}:{d:.2g}")
    print(f"{tag}: loss {tr.last_loss():.6f} (eager {ref_loss:.6f}) drifted: {len(bad)} {bad[:12]}", flush=True)
    return not bad


ok = check("replay1 vs eager")
for i in range(3):
    tr.step()
    ok &= check(f"replay{i + 2}")
junk = torch.full((512 * 2**20,), float("nan"), device="cuda")
del junk
tr.step()
ok &= check("after freed NaN alloc")
keep = [torch.full((64 * 2**20,), float("nan"), device="cuda") for _ in range(8)]
tr.step()
ok &= check("with NaN allocs live")
print("GRAPH_OK" if ok else "GRAPH_DRIFT")
sys.exit(0 if ok else 1)
