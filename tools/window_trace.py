#!/usr/bin/env python3
"""Where the time of bench.py's timed window goes, from one rocprofv3 run
with ``--kernel-trace --hip-runtime-trace --output-format csv``.

The timed window of the N=1 bench is ``sync -> run(K) -> sync``: the last
``hipGraphLaunch`` call(s) before the final ``hipDeviceSynchronize``.  This
prints, on one clock (ns from the profiler):

* host: launch-call begin -> end (submit time of the graph);
* launch-call begin -> first kernel of the window starts (GPU start lag);
* kernel busy time, idle gaps between the window's kernels;
* last kernel end -> synchronize returns (wake-up lag).

Usage: python tools/window_trace.py <dir with *_kernel_trace.csv and
*_hip_api_trace.csv> [--launches 1]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re


def _rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def _short(name: str) -> str:
    m = re.search(r"(k_[a-z0-9_]+)", name)
    return m.group(1) if m else name[:40]


def analyse(kernel_csv: str, api_csv: str, launches: int = 1) -> dict:
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), _short(r["Kernel_Name"]))
                for r in _rows(kernel_csv))
    api = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in _rows(api_csv))
    syncs = [a for a in api if a[2] in ("hipDeviceSynchronize", "hipStreamSynchronize")]
    launch = [a for a in api if a[2] in ("hipGraphLaunch", "hipGraphLaunch_spt")]
    if not launch:
        raise SystemExit("no hipGraphLaunch in the API trace")
    # the window = the last `launches` graph launches; its closing sync = the
    # first synchronize that begins after the last of them
    win = launch[-launches:]
    t_begin, t_submit_end = win[0][0], win[-1][1]
    end_sync = next((s for s in syncs if s[0] >= win[-1][0]), None)
    # the sync right before the window (bench's pre-window synchronize)
    pre_sync = max((s for s in syncs if s[1] <= t_begin), default=None, key=lambda s: s[1])
    kw = [k for k in ks if k[0] >= t_begin and (end_sync is None or k[1] <= end_sync[1])]
    if not kw:
        raise SystemExit("no kernels inside the window")
    busy = sum(e - s for s, e, _ in kw)
    gaps = [kw[i][0] - kw[i - 1][1] for i in range(1, len(kw))]
    big = sorted(((g, i) for i, g in enumerate(gaps, 1)), reverse=True)[:8]
    us = 1e-3
    out = {
        "kernels": len(kw),
        "graph_launch_calls": len(win),
        "pre_sync_end_to_launch_us": round((t_begin - pre_sync[1]) * us, 2) if pre_sync else None,
        "launch_call_us": round((t_submit_end - t_begin) * us, 2),
        "launch_to_first_kernel_us": round((kw[0][0] - t_begin) * us, 2),
        "kernel_busy_us": round(busy * us, 2),
        "gap_total_us": round(sum(gaps) * us, 2),
        "largest_gaps_us": [(round(g * us, 2), i, kw[i][2]) for g, i in big],
        "first_kernel_to_last_end_us": round((kw[-1][1] - kw[0][0]) * us, 2),
        "last_kernel_to_sync_return_us": round((end_sync[1] - kw[-1][1]) * us, 2) if end_sync else None,
        "launch_to_sync_return_us": round((end_sync[1] - t_begin) * us, 2) if end_sync else None,
        "per_kernel_us": {},
    }
    agg: dict[str, list] = {}
    for s, e, n in kw:
        agg.setdefault(n, []).append((e - s) * us)
    out["per_kernel_us"] = {n: round(sum(v) / len(v), 2) for n, v in agg.items()}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--launches", type=int, default=1)
    a = ap.parse_args()
    kc = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    hc = glob.glob(os.path.join(a.dir, "**", "*hip_api_trace.csv"), recursive=True)
    if not kc or not hc:
        raise SystemExit(f"need *kernel_trace.csv and *hip_api_trace.csv under {a.dir}")
    print(json.dumps(analyse(kc[0], hc[0], a.launches), indent=1))


if __name__ == "__main__":
    main()
