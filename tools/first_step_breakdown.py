#!/usr/bin/env python3
"""Where the fused MNIST trainer's time to its first optimizer step goes
(one GPU, world 1): HIP/torch init, trainer construction (data upload,
weights, kernel library load), graph capture of every step graph vs one
eager step.  Prints one JSON line."""
import json
import os
import sys
import time

t0 = time.perf_counter()
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
t_import = time.perf_counter()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
torch.zeros(1, device=dev)
torch.cuda.synchronize()
t_init = time.perf_counter()
from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer  # noqa: E402

tr = FusedMnistTrainer(dev, batch_size=64, dataset_size=60000, seed=1)
torch.cuda.synchronize()
t_ctor = time.perf_counter()
tr._eager_step()
torch.cuda.synchronize()
t_eager1 = time.perf_counter()
tr._eager_step()
torch.cuda.synchronize()
t_eager2 = time.perf_counter()
tr.run(1)
torch.cuda.synchronize()
t_run1 = time.perf_counter()
tr.run(1)
torch.cuda.synchronize()
t_run2 = time.perf_counter()
print(json.dumps({"import_torch_s": round(t_import - t0, 3), "hip_init_s": round(t_init - t_import, 3),
                  "trainer_ctor_s": round(t_ctor - t_init, 3), "first_eager_step_s": round(t_eager1 - t_ctor, 4),
                  "second_eager_step_s": round(t_eager2 - t_eager1, 5),
                  "first_run1_with_capture_s": round(t_run1 - t_eager2, 3),
                  "graphs_captured": len(tr._graph_pow) + len(tr._graph_close),
                  "second_run1_s": round(t_run2 - t_run1, 5)}), flush=True)
