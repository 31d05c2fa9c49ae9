#!/usr/bin/env python3
"""bf16 transpose on the Llama-3-8B step's shapes: the register-transpose
kernel (``pto_transpose_bf16``, what ``ops.llm.transpose_into`` runs) vs
PyTorch's ``y.copy_(x.t())``.  Checks the kernel against ``x.t()`` and
prints one JSON line per shape: us per call and effective HBM bandwidth
(read + write bytes / time).  The LDS-tiled kernel it replaced measured
10-25% slower on every shape (profiles/transpose_r4.md).
Usage: python tools/transpose_bench.py [--reps 50]"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

# (rows, cols, what): 4 x 4096 tokens per rank; Llama-3-8B dims
SHAPES = [
    (16384, 4096, "activations X / dY of wo (dW K-contiguous)"),
    (16384, 28672, "dY of w13"),
    (6144, 4096, "wqkv -> W^T"),
    (4096, 4096, "wo -> W^T"),
    (28672, 4096, "w13 -> W^T"),
    (4096, 14336, "w2 -> W^T"),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    from pytorch_operator_1_amd.ops import _lib

    L = _lib.lib()
    dev = torch.device("cuda", 0)
    s = _lib.stream_ptr(dev)
    for rows, cols, what in SHAPES:
        x = torch.randn(rows, cols, device=dev).bfloat16()
        ref = x.t().contiguous()
        out = {"rows": rows, "cols": cols, "what": what}
        y = torch.empty(cols, rows, device=dev, dtype=torch.bfloat16)
        runs = {"pto": lambda: L.pto_transpose_bf16(x.data_ptr(), y.data_ptr(), rows, cols, cols, rows, s),
                "torch": lambda: y.copy_(x.t())}
        _lib.check(runs["pto"](), "pto_transpose_bf16")
        torch.cuda.synchronize()
        out["pto_exact"] = bool(torch.equal(y, ref))
        for key, fn in runs.items():
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.reps
            out[key + "_us"] = round(us, 1)
            out[key + "_TBps"] = round(4 * rows * cols / us / 1e6, 2)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
