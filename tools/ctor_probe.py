#!/usr/bin/env python3
"""Breakdown of FusedMnistTrainer's constructor time on a fresh process:
synthetic data (device generator, then again warm), the stock module init,
and the constructor itself with data passed in.  Prints one JSON line (s).
Usage: python tools/ctor_probe.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_operator_1_amd.models.mnist import MnistNet, synthetic_mnist  # noqa: E402
from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer  # noqa: E402

dev = torch.device("cuda", 0)
torch.zeros(1, device=dev)
torch.cuda.synchronize()
out = {}
t = time.time()
x, y = synthetic_mnist(60000, dev, seed=2)
torch.cuda.synchronize()
out["data_first_s"] = round(time.time() - t, 4)
t = time.time()
x2, y2 = synthetic_mnist(60000, dev, seed=3)
torch.cuda.synchronize()
out["data_warm_s"] = round(time.time() - t, 4)
t = time.time()
torch.manual_seed(1)
MnistNet()
out["module_init_s"] = round(time.time() - t, 4)
t = time.time()
from pytorch_operator_1_amd.ops import _lib  # noqa: E402
_lib.lib()
out["lib_load_s"] = round(time.time() - t, 4)
t = time.time()
tr = FusedMnistTrainer(dev, batch_size=64, data=x.view(-1, 784), target=y)
torch.cuda.synchronize()
out["ctor_with_data_s"] = round(time.time() - t, 4)
print(json.dumps(out))
