#!/usr/bin/env python3
"""Deterministic-mode resume: per-parameter max |diff| between an
uninterrupted run and a run resumed from a step-4 state_dict, after each of
the next steps (debug aid for tests/test_graph_gpu.py)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("PTO_DETERMINISTIC", "1")
from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer  # noqa: E402

dev = torch.device("cuda", 0)
kw = dict(batch_size=64, dataset_size=64 * 9, seed=4, unroll=4)
c = FusedMnistTrainer(dev, **kw)
c.run(4)
sd = c.state_dict()
for k in range(1, 7):
    a = FusedMnistTrainer(dev, **kw)
    a.run(4 + k)
    a.flush()
    d = FusedMnistTrainer(dev, **kw)
    d.load_state_dict(sd)
    d.run(k)
    d.flush()
    torch.cuda.synchronize()
    diffs = {n: float((a.p[n] - d.p[n]).abs().max()) for n in a.p}
    print(k, {n: f"{v:.3g}" for n, v in diffs.items()}, "mom", f"{float((a.mom - d.mom).abs().max()):.3g}", flush=True)
a = FusedMnistTrainer(dev, **kw)
a.run(4)
a.flush()
torch.cuda.synchronize()
print("flushed-at-4 vs state_dict", {n: float((a.p[n] - sd['model'][n].to(dev)).abs().max()) for n in a.p})
