#!/usr/bin/env python3
"""What a kernel boundary costs vs a grid-wide barrier inside one kernel.

Per-kernel cost = host time of one replay of a graph of N identical
launches / N (sync -> replay -> sync, median).  Grid barrier cost =
(t(R rounds) - t(0 rounds)) / R for one launch of k_gridbar.  Decides
whether a persistent multi-phase kernel could beat launch boundaries for
the latency-bound MNIST step.  Usage: python tools/kernel_floor_probe.py"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    from pytorch_operator_1_amd.ops import _lib

    L = _lib.lib()
    dev = torch.device("cuda", 0)
    out = torch.zeros(1 << 20, device=dev)
    ctr = torch.zeros(2, dtype=torch.int32, device=dev)

    def timed(fn, reps=50):
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        return ts[len(ts) // 2] * 1e6

    def graph_of(launch, n):
        s = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            launch(s.cuda_stream)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(n):
                launch(torch.cuda.current_stream(dev).cuda_stream)
        g.replay()
        torch.cuda.synchronize()
        return g

    res = {}
    N = 40
    cases = {
        "noop_1x64": lambda st: L.pto_noop(1, st),
        "probe_128x1024": lambda st: L.pto_probe_kernel(128, 1024, None, 0, 0, st),
        "probe_256x1024": lambda st: L.pto_probe_kernel(256, 1024, None, 0, 0, st),
        "probe_256x1024_lds4": lambda st: L.pto_probe_kernel(256, 1024, None, 0, 4, st),
        "probe_128x1024_store128k": lambda st: L.pto_probe_kernel(128, 1024, _lib.ptr(out), 32768, 1, st),
        "probe_256x1024_store1m": lambda st: L.pto_probe_kernel(256, 1024, _lib.ptr(out), 262144, 1, st),
        "probe_256x256": lambda st: L.pto_probe_kernel(256, 256, None, 0, 0, st),
    }
    base1 = timed(graph_of(cases["noop_1x64"], 1).replay)
    res["graph_1_noop_us"] = round(base1, 2)
    for name, fn in cases.items():
        g = graph_of(fn, N)
        res[name + "_us_per_launch"] = round((timed(g.replay) - base1) / (N - 1), 3)
        print(json.dumps({name: res[name + "_us_per_launch"]}), flush=True)
    for blocks, threads in ((256, 64), (256, 1024), (128, 1024)):
        ts = {}
        for rounds in (0, 40):
            def one(st, rounds=rounds):
                ctr.zero_()
                return L.pto_gridbar_probe(blocks, threads, _lib.ptr(ctr), rounds, 200000, st)
            ts[rounds] = timed(lambda: one(torch.cuda.current_stream(dev).cuda_stream))
        fail = int(ctr[1].item())
        res[f"gridbar_{blocks}x{threads}_us_per_barrier"] = round((ts[40] - ts[0]) / 40, 3)
        res[f"gridbar_{blocks}x{threads}_timeouts"] = fail
        print(json.dumps({f"gridbar_{blocks}x{threads}": res[f"gridbar_{blocks}x{threads}_us_per_barrier"],
                          "timeouts": fail}), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
