#!/usr/bin/env python3
"""Why the driver's short bench window (--steps 20 --warmup 5) reads slower
than the steady-state step: the timed region of bench.py (sync -> run(20)
-> flush -> sync) repeated back to back right after a bench-like warmup,
then after idle gaps.  Usage: python tools/bench_window_probe.py
[--mode first|rewarm|rewarm_last] (first: only the first window after a
bench-like warmup; rewarm: every captured graph replayed twice more, state
rolled back, before the warmup steps; rewarm_last: the timed graph replayed
once more (rolled back) right before the window; upload_last: hipGraphUpload of the
timed graph right before the window)."""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="all", choices=["all", "first", "rewarm", "rewarm_last", "upload_last"])
    a = ap.parse_args()
    from pytorch_operator_1_amd.train.runner import build_trainer

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr = build_trainer("fused", device=dev, batch_size=64, lr=0.01, momentum=0.5, dataset_size=60000, seed=1)

    def window(n=20):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        tr.run(n)
        t1 = time.perf_counter()
        tr.flush()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        return round((t2 - t0) * 1e6, 1), round((t1 - t0) * 1e6, 1)

    def replay_rollback(graphs, times):
        state = tr._state()
        snap = [t.clone() for t in state]
        for _ in range(times):
            for g in graphs:
                g.replay()
        torch.cuda.synchronize(dev)
        for d, s_ in zip(state, snap):
            d.copy_(s_)
        torch.cuda.synchronize(dev)

    t0 = time.perf_counter()
    if a.mode == "rewarm":
        tr._ensure_captured()
        replay_rollback(list(tr._graph_pow.values()) + list(tr._graph_close.values()), 2)
    tr.run(5)
    if a.mode == "rewarm_last":
        replay_rollback([tr._graph_close[20]], 1)
    if a.mode == "upload_last":
        from pytorch_operator_1_amd.ops import _lib

        _lib.check(_lib.lib().pto_graph_upload(tr._graph_close[20].raw_cuda_graph_exec(), _lib.stream_ptr(dev)),
                   "hipGraphUpload")
    torch.cuda.synchronize(dev)
    out = {"mode": a.mode, "warmup_s": round(time.perf_counter() - t0, 2)}
    if a.mode != "all":
        out["first_windows"] = [window()]
        print(json.dumps(out))
        return
    out["back_to_back"] = [window() for _ in range(6)]
    for gap in (0.01, 0.1, 0.5):
        res = []
        for _ in range(3):
            time.sleep(gap)
            res.append(window())
        out[f"after_{gap}s_idle"] = res
    # a busy device right before the window (200 steps, untimed)
    res = []
    for _ in range(3):
        tr.run(200)
        res.append(window())
    out["after_200_steps"] = res
    print(json.dumps(out))


if __name__ == "__main__":
    main()
