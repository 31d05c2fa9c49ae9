#!/usr/bin/env python3
"""Per-kernel summary of the LAST N training steps of a rocprofv3 trace
(steps delimited by a marker kernel, e.g. the optimizer launch), so
warmup-time work (MIOpen find, lazy init) is excluded.

Usage: python tools/rocprof_window.py <db|dir> --marker sgd --steps 3 [--top 30]
"""
from __future__ import annotations

import argparse
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from rocprof_summary import load  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("path")
    p.add_argument("--marker", required=True, help="substring of the kernel that ends each step")
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--top", type=int, default=30)
    p.add_argument("--seq", action="store_true", help="also list the last step's dispatches in order")
    a = p.parse_args()
    import sqlite3
    import glob

    path = a.path
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(path)
    rows = list(c.execute("select name, start, end from kernels order by start"))
    marks = [i for i, r in enumerate(rows) if a.marker in r[0]]
    if len(marks) < a.steps + 1:
        raise SystemExit(f"only {len(marks)} marker kernels")
    lo, hi = marks[-a.steps - 1] + 1, marks[-1] + 1
    win = rows[lo:hi]
    agg = defaultdict(lambda: [0, 0.0])
    for name, s, e in win:
        agg[name][0] += 1
        agg[name][1] += e - s
    busy = sum(v[1] for v in agg.values())
    wall = win[-1][2] - win[0][1]
    print(f"window: last {a.steps} steps, {len(win)} dispatches, wall {wall / 1e6 / a.steps:.2f} ms/step, "
          f"kernel busy {busy / 1e6 / a.steps:.2f} ms/step\n")
    print("| kernel | calls/step | ms/step | % busy |")
    print("|---|---:|---:|---:|")
    for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        nm = name if len(name) <= 100 else name[:100] + "…"
        print(f"| `{nm}` | {n / a.steps:.1f} | {t / 1e6 / a.steps:.3f} | {100 * t / busy:.1f} |")
    if a.seq:  # the last step in dispatch order: who runs next to whom
        print("\n| # | kernel | us | gap before (us) |\n|---:|---|---:|---:|")
        last = rows[marks[-2] + 1:marks[-1] + 1]
        prev_end = last[0][1]
        for i, (name, s, e) in enumerate(last):
            print(f"| {i} | `{name[:90]}` | {(e - s) / 1e3:.1f} | {(s - prev_end) / 1e3:.1f} |")
            prev_end = e


if __name__ == "__main__":
    main()
