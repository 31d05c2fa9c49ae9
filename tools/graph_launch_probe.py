#!/usr/bin/env python3
"""Host-timed cost of replaying the fused trainer's captured step graphs
(sync -> replay -> sync, median of repeats): t(n) for the closing graph of
n steps, and split launches (a short graph first, so the GPU starts while
the rest is being submitted).  Usage: python tools/graph_launch_probe.py"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer

    dev = torch.device("cuda", 0)
    tr = FusedMnistTrainer(dev, batch_size=64, dataset_size=60000)
    tr.run(64)
    torch.cuda.synchronize()
    G, C = tr._graph_pow, tr._graph_close

    def timed(fn, reps=60):
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        return round(ts[len(ts) // 2] * 1e6, 2)

    ev = torch.cuda.Event()

    def spin_timed(fn, reps=60):
        # host waits by polling an event (no blocking wait), then synchronizes
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            ev.record()
            while not ev.query():
                pass
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        return round(ts[len(ts) // 2] * 1e6, 2)

    out = {}
    out["C20_spin"] = spin_timed(C[20].replay)
    out["C1_spin"] = spin_timed(C[1].replay)
    out["sync_only"] = timed(lambda: None)
    out["spin_only"] = spin_timed(lambda: None)
    for n in (1, 2, 4, 8, 16, 20, 32):
        out[f"C{n}"] = timed(C[n].replay)
    out["G1+C19"] = timed(lambda: (G[1].replay(), C[19].replay()))
    out["C1+C1"] = timed(lambda: (C[1].replay(), C[1].replay()))
    out["G32x2"] = timed(lambda: (G[32].replay(), G[32].replay()))
    out["C32+C32"] = timed(lambda: (C[32].replay(), C[32].replay()))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
