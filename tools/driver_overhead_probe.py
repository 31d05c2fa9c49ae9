"""Where the driver command's fixed cost goes (MNIST, one GPU).

``python bench.py --steps 20`` times one replay of the 20-step closing graph
plus the synchronisations around it; against the 2000-step steady state it
carries ~30 us of fixed cost (profiles/mnist_step_pmc_r6.md).  This probe
splits it: the host time of an empty ``torch.cuda.synchronize()``, a one-
kernel graph's replay-to-sync round trip, ``run(n)`` for several n (the
intercept of time vs n is the fixed cost), and the host time until
``replay()`` returns.  ``--spin`` sets ``hipDeviceScheduleSpin`` before the
runtime starts (the device-flag experiment).  Prints one JSON line.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spin", action="store_true")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    if a.spin:
        hip = ctypes.CDLL("libamdhip64.so")
        rc = hip.hipSetDeviceFlags(ctypes.c_uint(1))  # hipDeviceScheduleSpin
        print(f"[probe] hipSetDeviceFlags(spin) -> {rc}", file=sys.stderr)
    import torch

    from pytorch_operator_1_amd.train.runner import build_trainer

    dev = torch.device("cuda", 0)
    sync = torch.cuda.synchronize
    out = {"spin": a.spin}

    def make():
        return build_trainer("fused", device=dev, batch_size=64, lr=0.01, momentum=0.5, dataset_size=60000, seed=1,
                             rank=0)

    # bench.py's sequence: warm-up run(5) (captures every graph first),
    # prepare(), then the timed run(20) -- the first replay of the 20-step
    # closing graph since its capture; then the same run again, and again
    seq = []
    for _ in range(2):
        tr = make()
        tr.run(a.warmup)
        tr.prepare() if hasattr(tr, "prepare") else None
        ts = []
        for _ in range(5):
            sync()
            t0 = time.perf_counter()
            tr.run(20)
            tr.flush()
            sync()
            ts.append(round((time.perf_counter() - t0) * 1e6, 1))
        seq.append(ts)
        del tr
    out["bench_like_run20_us"] = seq
    # an idle GPU before the region: run(20) after the host sleeps (warm-up
    # steps then region, as bench.py does), per idle time
    tr = make()
    tr.run(a.warmup)
    tr.prepare() if hasattr(tr, "prepare") else None
    idle = {}
    for rep in range(3):
        for ms in (0, 2, 20, 200, 1000):
            sync()
            time.sleep(ms / 1e3)
            tr.run(a.warmup)
            sync()
            t0 = time.perf_counter()
            tr.run(20)
            tr.flush()
            sync()
            idle.setdefault(ms, []).append(round((time.perf_counter() - t0) * 1e6, 1))
    out["after_idle_ms_run20_us"] = idle
    # what the replay just before the region does to it
    x = torch.zeros(1, device=dev)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        x.add_(1)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            x.add_(1)
    g.replay()
    sync()
    before = {"run20": lambda: tr.run(20), "run5": lambda: tr.run(5), "run1": lambda: tr.run(1),
              "run32": lambda: tr.run(32), "tiny_graph": g.replay, "tiny_kernel": lambda: x.add_(1),
              "nothing": lambda: None}
    prev = {}
    for rep in range(4):
        for name, f in before.items():
            sync()
            f()
            sync()
            t0 = time.perf_counter()
            tr.run(20)
            sync()
            prev.setdefault(name, []).append(round((time.perf_counter() - t0) * 1e6, 1))
    out["run20_after_us"] = prev
    del tr
    tr = make()
    tr.run(1)
    tr.run(5)
    tr.prepare() if hasattr(tr, "prepare") else None
    sync()

    def med(f, reps=a.reps):
        ts = []
        for _ in range(reps):
            sync()
            t0 = time.perf_counter()
            f()
            ts.append((time.perf_counter() - t0) * 1e6)
        return round(statistics.median(ts), 2), round(min(ts), 2)

    out["sync_empty_us"] = med(sync)
    x = torch.zeros(1, device=dev)
    out["tiny_kernel_sync_us"] = med(lambda: (x.add_(1), sync()))
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        x.add_(1)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            x.add_(1)
    g.replay()
    out["tiny_graph_sync_us"] = med(lambda: (g.replay(), sync()))
    runs = {}
    for n in (1, 2, 4, 8, 16, 20, 32):
        runs[n] = med(lambda: (tr.run(n), tr.flush(), sync()))[0]
    out["run_us"] = runs
    ns = sorted(runs)
    mx, my = statistics.mean(ns), statistics.mean(runs[n] for n in ns)
    slope = sum((n - mx) * (runs[n] - my) for n in ns) / sum((n - mx) ** 2 for n in ns)
    out["fit_us_per_step"] = round(slope, 3)
    out["fit_fixed_us"] = round(my - slope * mx, 2)
    out["run20_minus_20x_slope_us"] = round(runs[20] - 20 * slope, 2)
    rets = []
    for _ in range(a.reps):
        sync()
        t0 = time.perf_counter()
        tr.run(20)
        t1 = time.perf_counter()
        sync()
        rets.append((t1 - t0) * 1e6)
    out["run20_return_us"] = round(statistics.median(rets), 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
