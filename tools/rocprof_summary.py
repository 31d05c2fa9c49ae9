#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--kernel-trace`` output (rocpd SQLite ``.db`` or
``kernel_trace.csv``) into a markdown table: per-kernel calls, total/avg
time, share, plus VGPR/LDS/grid of the dispatch.

Usage: python tools/rocprof_summary.py <db|csv|dir> [--steps N] [--top K]
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import sqlite3
from collections import defaultdict


def _rows_from_db(path):
    c = sqlite3.connect(path)
    cur = c.execute(
        "select name, duration, grid_x, workgroup_x, vgpr_count, accum_vgpr_count, lds_size from kernels")
    for name, dur, gx, wx, vg, ag, lds in cur:
        yield name, float(dur), int(gx or 0), int(wx or 0), int(vg or 0), int(ag or 0), int(lds or 0)


def _rows_from_csv(path):
    with open(path) as f:
        for r in csv.DictReader(f):
            dur = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            yield (r["Kernel_Name"], dur, int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0),
                   int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 0)) or 0), int(r.get("VGPR_Count", 0) or 0),
                   int(r.get("Accum_VGPR_Count", 0) or 0), int(r.get("LDS_Block_Size", 0) or 0))


def load(path):
    if os.path.isdir(path):
        cands = glob.glob(os.path.join(path, "**", "*.db"), recursive=True) + \
            glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
        if not cands:
            raise SystemExit(f"no .db / kernel_trace.csv under {path}")
        path = cands[0]
    return list(_rows_from_db(path) if path.endswith(".db") else _rows_from_csv(path)), path


def summarise(rows, steps=None, top=30, short=90):
    agg = defaultdict(lambda: [0, 0.0, None])
    for name, dur, gx, wx, vg, ag, lds in rows:
        a = agg[name]
        a[0] += 1
        a[1] += dur
        a[2] = (gx, wx, vg, ag, lds)
    total = sum(a[1] for a in agg.values())
    lines = ["| kernel | calls | total us | avg us | % | grid | wg | vgpr | agpr | lds |",
             "|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|"]
    for name, (n, t, meta) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        nm = name if len(name) <= short else name[:short] + "…"
        gx, wx, vg, ag, lds = meta
        lines.append(f"| `{nm}` | {n} | {t / 1e3:.1f} | {t / n / 1e3:.2f} | {100 * t / total:.1f} | {gx} | {wx} | "
                     f"{vg} | {ag} | {lds} |")
    head = [f"total kernel time: {total / 1e3:.1f} us over {sum(a[0] for a in agg.values())} dispatches"]
    if steps:
        head.append(f"per step ({steps} steps): {total / 1e3 / steps:.2f} us kernel time, "
                    f"{sum(a[0] for a in agg.values()) / steps:.1f} dispatches")
    return "\n".join(head + [""] + lines)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("path")
    p.add_argument("--steps", type=int, default=None)
    p.add_argument("--top", type=int, default=30)
    a = p.parse_args()
    rows, path = load(a.path)
    print(f"source: `{os.path.basename(path)}`\n")
    print(summarise(rows, a.steps, a.top))


if __name__ == "__main__":
    main()
