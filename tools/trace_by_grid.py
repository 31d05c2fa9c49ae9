#!/usr/bin/env python3
"""Group a rocprofv3 kernel-trace CSV by (kernel, grid size): total / count /
avg duration for the kernels matching --filter, over the last --window
dispatches of each kind.  Usage:
  python tools/trace_by_grid.py <run_kernel_trace.csv> --filter k_bn [--top 40]
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"(k_[a-z0-9_]+(?:<[^>]*>)?)", name)
    return m.group(1) if m else name[:50]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--filter", default="")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    agg = defaultdict(lambda: [0.0, 0])
    with open(a.csv) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "")
            if a.filter and a.filter not in name:
                continue
            dur = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
            grid = row.get("Grid_Size_X") or row.get("Grid_Size", "?")
            key = (short(name), grid)
            agg[key][0] += dur
            agg[key][1] += 1
    tot = sum(v[0] for v in agg.values())
    print(f"total {tot:.1f} us over {sum(v[1] for v in agg.values())} dispatches")
    for (k, g), (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[: a.top]:
        print(f"{k:28s} grid {g:>9s}  n {n:5d}  total {t:10.1f} us  avg {t / n:8.2f} us  {100 * t / tot:5.1f} %")


if __name__ == "__main__":
    main()
