#!/usr/bin/env python3
"""Per-shape time and HBM bandwidth of the fused BN kernels from a rocprofv3
database of ``tools/bn_bench.py`` (``rocprofv3 --kernel-trace -o bn -- python3
tools/bn_bench.py``).  bn_bench runs its shapes in order and every kernel the
same number of times per shape, so a kernel's dispatches split evenly into
per-shape groups.  Prints one line per (kernel, shape): median us and TB/s
(bytes = passes x activation bytes).
Usage: python tools/bn_kernel_table.py gpurun_out/bn/prof/bn_results.db"""
import collections
import sqlite3
import sys

SHAPES = [(64, 112), (64, 56), (256, 56), (128, 28), (512, 28), (1024, 14), (2048, 7)]
# full-tensor passes per kernel (bf16 activation streams read + written)
PASSES = {"k_bn_stats": 1, "k_bn_apply<false, true>": 2, "k_bn_bwd_reduce<1>": 2, "k_bn_bwd_apply<1>": 3}


def main(db: str):
    con = sqlite3.connect(db)
    seq = collections.defaultdict(list)
    for name, dur in con.execute("select name, duration from kernels order by start"):
        k = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        if k in PASSES:
            seq[k].append(dur / 1000.0)
    for k, v in seq.items():
        per = len(v) // len(SHAPES)
        for i, (C, HW) in enumerate(SHAPES):
            c = sorted(v[i * per:(i + 1) * per])
            med = c[len(c) // 2]
            mb = 256 * C * HW * HW * 2 / 1e6
            print(f"{k:26s} C={C:5d} HW={HW:4d} {mb:6.0f} MB  {med:8.1f} us  {PASSES[k] * mb / med:5.2f} TB/s")


if __name__ == "__main__":
    main(sys.argv[1])
