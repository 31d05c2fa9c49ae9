#!/usr/bin/env python3
"""What bounds the short timed window at N=1 besides the kernels: the
host wait at the end (HIP device flags: default / spin / yield / blocking
sync) and the GPU start at the beginning (a graph launch vs direct kernel
launches for the first step, the rest as one graph).  Host-timed
sync -> work -> sync windows, median of repeats, on the fused trainer.
Usage: python tools/sync_latency_probe.py"""
from __future__ import annotations

import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

FLAGS = {"auto": 0, "spin": 1, "yield": 2, "blocking": 4}


def main():
    from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer

    dev = torch.device("cuda", 0)
    tr = FusedMnistTrainer(dev, batch_size=64, dataset_size=60000)
    tr.run(64)
    torch.cuda.synchronize()
    hip = ctypes.CDLL("libamdhip64.so")
    C = tr._graph_close

    def timed(fn, reps=40):
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        return round(ts[len(ts) // 2] * 1e6, 2)

    def eager_head_then(n):
        def f():
            tr._forward()
            tr._backward()
            C[n - 1].replay()
        return f

    out = {}
    for name, fl in FLAGS.items():
        rc = hip.hipSetDeviceFlags(ctypes.c_uint(fl))
        cur = ctypes.c_uint(0)
        hip.hipGetDeviceFlags(ctypes.byref(cur))
        r = {"rc": rc, "flags": cur.value}
        r["sync_idle"] = timed(lambda: None)
        r["noop"] = timed(lambda: tr.L.pto_noop(1, tr._s()))
        r["C1"] = timed(C[1].replay)
        r["C20"] = timed(C[20].replay)
        r["eager1+C19"] = timed(eager_head_then(20))
        out[name] = r
    hip.hipSetDeviceFlags(ctypes.c_uint(0))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
