#!/usr/bin/env python3
"""Gradient all-reduce sweep + Llama-3-8B bucket stress (SURVEY §7.2 step 9,
BASELINE config 4 "grad-bucket all-reduce stress").

One process per GPU under ``torch.distributed.run``::

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        tools/allreduce_bench.py --sizes-mb 0.1,1.7,16,256 --stress-gb 16

* sweep: RCCL all-reduce (and the xGMI peer kernel for fp32 buckets up to
  ``--xgmi-max-mb``) per message size; time per call (max over ranks),
  algorithm bandwidth = bytes / t and bus bandwidth = algbw * 2 (n-1) / n
  (what a ring moves per GPU: the number to compare against the 7 xGMI
  links of one MI355X);
* stress: ``--stress-gb`` of bf16 gradients (Llama-3-8B: 16 GB) as
  ``--bucket-mb`` buckets issued back to back on a comm stream, exactly as
  :class:`~pytorch_operator_1_amd.parallel.ddp.GradBucketer` does during
  backward, then every bucket is checked against the expected sum.

Rank 0 prints one JSON line per measurement.  ``--cpu`` runs gloo on CPU
(plumbing check only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _max(v: float, dev) -> float:
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def timed(fn, iters: int, dev) -> float:
    fn()
    _sync(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    _sync(dev)
    return _max((time.perf_counter() - t0) / iters, dev)


def sweep(sizes_mb, dtype, iters, dev, xgmi_max_mb, out):
    n = dist.get_world_size()
    esz = torch.empty((), dtype=dtype).element_size()
    xgmi = None
    for mb in sizes_mb:
        numel = max(4, int(mb * 2**20 / esz) // 4 * 4)
        buf = torch.ones(numel, dtype=dtype, device=dev)
        t = timed(lambda: dist.all_reduce(buf), iters, dev)
        nbytes = numel * esz
        rec = {"op": "all_reduce", "impl": dist.get_backend(), "dtype": str(dtype).split(".")[-1], "bytes": nbytes,
               "us": round(t * 1e6, 2), "algbw_GBps": round(nbytes / t / 1e9, 2),
               "busbw_GBps": round(nbytes / t / 1e9 * 2 * (n - 1) / n, 2), "world": n}
        out(rec)
        if dev.type == "cuda" and dtype == torch.float32 and mb <= xgmi_max_mb and n > 1:
            from pytorch_operator_1_amd.parallel.xgmi import XgmiAllReduce

            if xgmi is not None:
                xgmi.close()
            try:
                xgmi = XgmiAllReduce(buf)
            except (RuntimeError, ValueError) as e:
                out({"op": "all_reduce", "impl": "xgmi", "error": str(e)[:200]})
                xgmi = None
                continue
            t = timed(lambda: xgmi.allreduce_(0, numel), iters, dev)
            xgmi.check()
            out(dict(rec, impl="xgmi", us=round(t * 1e6, 2), algbw_GBps=round(nbytes / t / 1e9, 2),
                     busbw_GBps=round(nbytes / t / 1e9 * 2 * (n - 1) / n, 2)))
    if xgmi is not None:
        xgmi.close()


def stress(total_gb, bucket_mb, dev, out):
    """Back-to-back bucket all-reduces on a comm stream, then verification."""
    n, r = dist.get_world_size(), dist.get_rank()
    esz = 2
    per = int(bucket_mb * 2**20 / esz)
    nb = max(1, int(total_gb * 2**30 / (per * esz)))
    # one flat buffer like GradBucketer's; rank r's gradients = r + 1, so the
    # SUM is n (n + 1) / 2 everywhere (exact in bf16 for n <= 8)
    flat = torch.full((nb * per,), float(r + 1), dtype=torch.bfloat16, device=dev)
    stream = torch.cuda.Stream(dev) if dev.type == "cuda" else None
    _sync(dev)
    dist.barrier()
    t0 = time.perf_counter()
    works = []
    for i in range(nb):
        view = flat[i * per:(i + 1) * per]
        if stream is not None:
            ev = torch.cuda.current_stream(dev).record_event()
            stream.wait_event(ev)
            with torch.cuda.stream(stream):
                works.append(dist.all_reduce(view, async_op=True))
        else:
            works.append(dist.all_reduce(view, async_op=True))
    for w in works:
        w.wait()
    if stream is not None:
        torch.cuda.current_stream(dev).wait_stream(stream)
    _sync(dev)
    t = _max(time.perf_counter() - t0, dev)
    want = float(n * (n + 1) // 2)
    bad = int((flat != want).sum().item())
    bad = int(_max(float(bad), dev))
    nbytes = nb * per * esz
    out({"op": "bucket_stress", "impl": dist.get_backend(), "buckets": nb, "bucket_mb": bucket_mb,
         "total_gb": round(nbytes / 2**30, 2), "s": round(t, 4), "algbw_GBps": round(nbytes / t / 1e9, 2),
         "busbw_GBps": round(nbytes / t / 1e9 * 2 * (n - 1) / n, 2), "mismatched_elements": bad, "world": n})
    return bad


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--sizes-mb", default="0.1,1.7,16,64,256")
    p.add_argument("--dtype", default="float32", choices=["float32", "bfloat16"])
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--xgmi-max-mb", type=float, default=64.0)
    p.add_argument("--stress-gb", type=float, default=0.0, help="bf16 gradient volume of the stress pass (0: skip)")
    p.add_argument("--bucket-mb", type=float, default=256.0)
    p.add_argument("--cpu", action="store_true")
    a = p.parse_args(argv)
    from pytorch_operator_1_amd.utils import dist as pdist

    use_gpu = torch.cuda.is_available() and not a.cpu
    env, dev = pdist.init_distributed(os.environ.get("PTO_BACKEND"), use_gpu=use_gpu)
    if not dist.is_initialized():
        raise SystemExit("run under torch.distributed.run (WORLD_SIZE >= 1)")

    def out(rec):
        if env.rank == 0:
            print(json.dumps(rec), flush=True)

    sweep([float(s) for s in a.sizes_mb.split(",") if s], getattr(torch, a.dtype), a.iters, dev, a.xgmi_max_mb, out)
    bad = stress(a.stress_gb, a.bucket_mb, dev, out) if a.stress_gb > 0 else 0
    pdist.cleanup()
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
