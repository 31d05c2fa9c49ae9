#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc runs (rocpd .db files): per kernel (name
filter), the counter totals per dispatch, averaged over dispatches.

Usage: python tools/pmc_summary.py <dir-or-db> [<dir-or-db> ...] --filter attn
"""
import argparse
import glob
import os
import re
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"(k_[a-z0-9_]+)", name)
    return m.group(1) if m else name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("paths", nargs="+")
    ap.add_argument("--filter", default="")
    ap.add_argument("--skip", type=int, default=0, help="drop each kernel's first N dispatches")
    ap.add_argument("--per-dispatch", action="store_true", help="one line per dispatch instead of averages")
    a = ap.parse_args()
    # kernel -> counter -> list of per-dispatch totals
    acc = defaultdict(lambda: defaultdict(list))
    for p in a.paths:
        dbs = glob.glob(os.path.join(p, "**", "*.db"), recursive=True) if os.path.isdir(p) else [p]
        for db in dbs:
            c = sqlite3.connect(db)
            per = defaultdict(float)
            for name, disp, ctr, val in c.execute(
                    "select name, dispatch_id, counter_name, counter_value from pmc_events"):
                if a.filter and a.filter not in name:
                    continue
                per[(short(name), disp, ctr)] += val
            if a.per_dispatch:
                rows = defaultdict(dict)
                for (k, d, ctr), v in per.items():
                    rows[(d, k)][ctr] = v
                for (d, k), cv in sorted(rows.items()):
                    print(f"{d:6d} {k[:40]:40s} " + "  ".join(f"{c}={v:.4g}" for c, v in sorted(cv.items())))
                continue
            first = defaultdict(list)
            for (k, d, ctr) in per:
                first[k].append(d)
            keep = {k: set(sorted(set(ds))[a.skip:]) for k, ds in first.items()}
            for (k, d, ctr), v in per.items():
                if d in keep[k]:
                    acc[k][ctr].append(v)
    for k, ctrs in acc.items():
        print(f"## {k}")
        for ctr, vals in sorted(ctrs.items()):
            print(f"  {ctr:28s} {sum(vals) / len(vals):16.4g}  (n={len(vals)})")


if __name__ == "__main__":
    main()
