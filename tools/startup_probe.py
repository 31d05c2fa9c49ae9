#!/usr/bin/env python3
"""Where a fused MNIST trainer's time to its first optimizer step goes, in
one process on one GPU: importing torch, HIP init, the trainer constructor
(buffers, init weights, synthetic data), the first run(1) (one eager step:
graph capture deferred), then the deferred capture of every step graph and
a replayed step.  Prints one JSON line (seconds).
Usage: python tools/startup_probe.py"""
import json
import os
import sys
import time

t0 = time.time()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

t1 = time.time()
from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer  # noqa: E402

dev = torch.device("cuda", 0)
torch.zeros(1, device=dev)
torch.cuda.synchronize()
t2 = time.time()
tr = FusedMnistTrainer(dev, batch_size=64, dataset_size=60000)
torch.cuda.synchronize()
t3 = time.time()
tr.run(1)  # the first optimizer step (eager launches)
torch.cuda.synchronize()
t4 = time.time()
tr.run(2)  # captures every step graph, then replays
torch.cuda.synchronize()
t5 = time.time()
tr.run(1)
torch.cuda.synchronize()
t6 = time.time()
print(json.dumps({"import_torch_s": round(t1 - t0, 3), "hip_init_s": round(t2 - t1, 3),
                  "trainer_ctor_s": round(t3 - t2, 3), "first_step_s": round(t4 - t3, 4),
                  "capture_plus_2_steps_s": round(t5 - t4, 3), "replayed_step_s": round(t6 - t5, 5)}))
