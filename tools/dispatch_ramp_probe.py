#!/usr/bin/env python3
"""Workgroup dispatch ramp (round 6, k_bwd_all analysis): for grids shaped
like the MNIST step's launches (and variants), how long after the first
block does the last block of the grid start, and when does the grid end?
Median over 20 launches of (last entry - first entry) and (last exit -
first entry), µs.  Usage: python tools/dispatch_ramp_probe.py [--build]"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tools", "probes", "dispatch_ramp.hip")
SO = os.path.join(ROOT, "tools", "probes", "libdispatch_ramp.so")

# (name, blocks, threads, dynamic LDS bytes)
SHAPES = [("k_bwd_all-like 1422 x 256, 30 KB", 1422, 256, 30400),
          ("1422 x 256, no LDS", 1422, 256, 0),
          ("1280 x 256, 30 KB (exactly resident)", 1280, 256, 30400),
          ("711 x 512, 60 KB", 711, 512, 60800),
          ("356 x 1024, 120 KB", 356, 1024, 121600),
          ("F12-like 256 x 1024, 60 KB", 256, 1024, 61232),
          ("F4dx-like 201 x 1024, 72 KB", 201, 1024, 73760)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--spin", type=int, default=20)
    a = ap.parse_args()
    if a.build:
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", SO, SRC])
        print("built", SO)
        return
    import torch

    lib = ctypes.CDLL(SO)
    lib.ramp_launch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    out = {}
    for name, blocks, threads, lds in SHAPES:
        st = torch.zeros(2 * blocks, dtype=torch.int64, device=dev)
        ramps, spans = [], []
        for _ in range(22):
            rc = lib.ramp_launch(st.data_ptr(), blocks, threads, lds, a.spin, torch.cuda.current_stream().cuda_stream)
            assert rc == 0, rc
            torch.cuda.synchronize()
            v = st.view(-1, 2).cpu()
            e0 = int(v[:, 0].min())
            ramps.append((int(v[:, 0].max()) - e0) / 100.0)  # 100 MHz ticks -> us
            spans.append((int(v[:, 1].max()) - e0) / 100.0)
        ramps, spans = sorted(ramps[2:]), sorted(spans[2:])
        out[name] = {"entry_spread_us": ramps[len(ramps) // 2], "span_us": spans[len(spans) // 2]}
        print(json.dumps({name: out[name]}), flush=True)


if __name__ == "__main__":
    main()
