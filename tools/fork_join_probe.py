#!/usr/bin/env python3
"""In-graph cost of a side-stream fork/join on the CURRENT MNIST step
(verdict r3: the 19 us figure in profiles/graph_fork_join_probe_r1.md is a
round-1 measurement on a 54 us step).

Captures 32 consecutive fused-opt steps three ways and replays each graph
(host-timed, median of repeats, us per step):
  plain      the shipped launch sequence (4 launches per step);
  fork       + one fork/join per step: after F4dx a side stream (waiting on
             the main stream) runs one tiny kernel, and the main stream waits
             for it before k_bwd_all;
  fork_late  the same branch joined only before the NEXT step's F12, so the
             side kernel can overlap k_bwd_all (the shape an overlapped
             exchange on a second stream would have).
With --ablate: also the step with ONE of its four launches left out
(no_F12 / no_F3 / no_F4dx / no_bwd), i.e. each launch's marginal cost inside
the replayed graph (the kernels then read stale activations: timing only).
Timing only: the trainer state is rolled back afterwards, numerics are not
checked.  Usage: python tools/fork_join_probe.py [--steps 32] [--reps 30]"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--ablate", action="store_true")
    a = ap.parse_args()
    from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer

    dev = torch.device("cuda", 0)
    tr = FusedMnistTrainer(dev, batch_size=64, dataset_size=60000)
    tr.run(8)
    torch.cuda.synchronize()
    snap = [t.clone() for t in tr._state()]
    main_s = torch.cuda.Stream(dev)
    side = torch.cuda.Stream(dev)
    tiny = torch.zeros(64, device=dev)

    def step(mode: str):
        if mode.startswith("no_"):
            for which, name in enumerate(("F12", "F3", "F4dx")):
                if mode != "no_" + name:
                    tr._forward(only=which)
            if mode != "no_bwd":
                tr._backward()
            return
        tr._forward()
        if mode == "plain":
            tr._backward()
            return
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            tiny.add_(1.0)
        if mode == "fork":
            torch.cuda.current_stream(dev).wait_stream(side)
            tr._backward()
        else:  # fork_late: joined after the backward, before the next F12
            tr._backward()
            torch.cuda.current_stream(dev).wait_stream(side)

    graphs = {}
    modes = ["plain", "fork", "fork_late"] + (["no_F12", "no_F3", "no_F4dx", "no_bwd"] if a.ablate else [])
    for mode in modes:
        with torch.cuda.stream(main_s):  # warm the branch outside capture
            step(mode)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=main_s):
            for _ in range(a.steps):
                step(mode)
        graphs[mode] = g
        g.replay()  # first replay uploads the graph
        torch.cuda.synchronize()

    def timed(g):
        ts = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g.replay()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        return ts[len(ts) // 2] * 1e6 / a.steps

    out = {"steps_per_graph": a.steps}
    for _ in range(2):  # interleaved, twice
        for mode, g in graphs.items():
            out.setdefault(mode + "_us_per_step", []).append(round(timed(g), 2))
    for d, s in zip(tr._state(), snap):
        d.copy_(s)
    torch.cuda.synchronize()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
