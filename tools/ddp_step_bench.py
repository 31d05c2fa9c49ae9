#!/usr/bin/env python3
"""Per-step time of the fused MNIST trainer's MULTI-GPU schedule at world
size 1 (``force_ddp``: grads-only backward, then either the RCCL
all-reduce of a 1-rank group + the multi-tensor SGD launch, or the xGMI
all-reduce kernel with its SGD epilogue over one rank -- the per-rank
launches of the N>1 step without the peer traffic), next to the one-process
fused-optimizer step.  Prints one JSON line.

Usage: python tools/ddp_step_bench.py [--steps 2000] [--warmup 200]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--only", choices=["ddp", "xgmi", "xgmi_noov", "single"], default=None,
                    help="time one schedule (for rocprof)")
    a = ap.parse_args()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer

    out = {}
    # ddp: grads-only step + RCCL all-reduce of the 1-rank group + SGD launch;
    # xgmi: grads-only step + the xGMI all-reduce kernel with its SGD
    # epilogue over one rank (the N>1 step's launches minus the peer reads)
    # xgmi: the fc part of the exchange inside the next step's F12 launch
    # (overlap, the default); xgmi_noov: one whole-buffer all-reduce per step
    runs = (("ddp_step_us", "ddp", dict(force_ddp=True, comm="rccl")),
            ("ddp_xgmi_step_us", "xgmi", dict(force_ddp=True, comm="xgmi")),
            ("ddp_xgmi_noov_step_us", "xgmi_noov", dict(force_ddp=True, comm="xgmi", overlap=False)),
            ("single_gpu_step_us", "single", {}))
    for key, tag, kw in runs:
        if a.only and a.only != tag:
            continue
        tr = FusedMnistTrainer(dev, batch_size=64, dataset_size=60000, **kw)
        tr.run(a.warmup)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.run(a.steps)
        torch.cuda.synchronize()
        out[key] = round((time.perf_counter() - t0) / a.steps * 1e6, 2)
        out[key.replace("_step_us", "_schedule")] = tr.schedule
        out[key.replace("_step_us", "_loss")] = round(tr.last_loss(), 4)
    print(json.dumps(out))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
