#!/usr/bin/env python3
"""Idle gaps between consecutive kernels in the last N dispatches of a
rocprofv3 kernel-trace CSV (is the GPU waiting for the host between
launches?).  Usage: python tools/trace_gaps.py <kernel_trace.csv> --last 81"""
import argparse
import csv
import re


def short(name: str) -> str:
    m = re.search(r"(k_[a-z0-9_]+)", name)
    return m.group(1) if m else name[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last", type=int, default=81)
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    rows = rows[-a.last:]
    gaps = []
    for i, (s, e, n) in enumerate(rows):
        gap = (s - rows[i - 1][1]) / 1e3 if i else 0.0
        gaps.append(gap)
        print(f"{i:4d} {n:28s} start {(s - rows[0][0]) / 1e3:9.2f} us  dur {(e - s) / 1e3:7.2f}  gap {gap:7.2f}")
    span = (rows[-1][1] - rows[0][0]) / 1e3
    busy = sum(e - s for s, e, _ in rows) / 1e3
    print(f"span {span:.1f} us, busy {busy:.1f} us, gaps {sum(gaps):.1f} us, max gap {max(gaps):.1f} us")


if __name__ == "__main__":
    main()
