#!/usr/bin/env python3
"""Headline benchmark: MNIST DDP training samples/sec (BASELINE.json).

Config (reference ``examples/mnist/mnist.py``): the reference ``Net``
(431,080 fp32 params), batch 64 per rank, SGD lr=0.01 momentum=0.5,
NLL loss on log-softmax, DDP gradient averaging, fp32 compute.  One
process per GPU; for N>1 the driver launches this file under
``torch.distributed.run`` and ranks talk RCCL (torch backend ``nccl``).

Weak scaling: per-rank batch is fixed at 64, ``value`` is the aggregate
samples/s over all ranks (reference-equivalent mode: no sampler, every
rank runs its own batch stream, exactly like the reference's mnist.py).

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--impl fused|eager]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

# Reference-derived per-rank throughput lower bound (60,000
# samples / 286 s on the CPU cluster, gloo, 2 ranks).
BASELINE_SAMPLES_PER_SEC_PER_RANK = 210.0


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=2000)
    p.add_argument("--warmup", type=int, default=200)
    p.add_argument("--batch-size", type=int, default=64)
    p.add_argument("--lr", type=float, default=0.01)
    p.add_argument("--momentum", type=float, default=0.5)
    p.add_argument("--impl", choices=["fused", "eager"], default=os.environ.get("BENCH_IMPL", "fused"))
    p.add_argument("--dataset-size", type=int, default=60000)
    p.add_argument("--cpu", action="store_true", help="run on CPU with gloo (debug only)")
    p.add_argument("--verbose", action="store_true")
    return p.parse_args(argv)


def main(argv=None):
    args = parse_args(argv)
    from pytorch_operator_1_amd.utils import dist as pdist

    use_gpu = torch.cuda.is_available() and not args.cpu
    env, device = pdist.init_distributed(use_gpu=use_gpu)
    if env.world_size != args.gpus and env.rank == 0:
        print(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE={env.world_size}", file=sys.stderr)

    from pytorch_operator_1_amd.train.runner import build_trainer

    trainer = build_trainer(args.impl, device=device, batch_size=args.batch_size, lr=args.lr,
                            momentum=args.momentum, dataset_size=args.dataset_size,
                            seed=1 + env.rank * 0, rank=env.rank)

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    for _ in range(args.warmup):
        trainer.step()
    sync()
    pdist.barrier(device)
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        trainer.step()
    sync()
    pdist.barrier(device)
    sync()
    elapsed = time.perf_counter() - t0
    elapsed = pdist.all_reduce_max(elapsed, device)
    loss = trainer.last_loss()

    n = env.world_size
    ms_per_step = elapsed / args.steps * 1e3
    value = args.batch_size * n * args.steps / elapsed
    if env.rank == 0:
        out = {
            "metric": "samples/sec MNIST DDP",
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / (BASELINE_SAMPLES_PER_SEC_PER_RANK * n), 1),
            "dtype": "fp32",
            "data": "synthetic (MNIST-shaped 1x28x28, resident in HBM), random-init weights",
            "config": {
                "model": "mnist-cnn (reference examples/mnist/mnist.py Net, 431,080 params)",
                "global_batch": args.batch_size * n,
                "per_rank_batch": args.batch_size,
                "seq_len": None,
                "input_shape": [1, 28, 28],
                "optimizer": f"SGD lr={args.lr} momentum={args.momentum}",
                "parallelism": f"dp{n}",
                "impl": args.impl,
                "backend": (torch.distributed.get_backend() if n > 1 else "none"),
                "baseline": "210 samples/s/rank (BASELINE.md, derived lower bound); vs_baseline = value/(210*n_gpus)",
                "final_loss": round(loss, 4) if loss is not None else None,
            },
        }
        print(json.dumps(out), flush=True)
    pdist.cleanup()


if __name__ == "__main__":
    main()
