#!/usr/bin/env python3
"""Per-launch timing of the fused MNIST step kernels (one process, HIP
events, median over interleaved rounds — cdna_hip_programming.md §5.4
rule 24).  Usage: python tools/kernel_bench.py [--iters 200] [--json out]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from pytorch_operator_1_amd.ops import _lib
    from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer

    dev = torch.device("cuda", 0)
    # the DDP schedule's launches are pure functions of the trainer's buffers
    # (grads-only backward: no parameter changes), so each can be re-timed
    tr = FusedMnistTrainer(dev, batch_size=a.batch, dataset_size=a.batch * 16, graph="none", force_ddp=True)
    for _ in range(5):
        tr.step()
    torch.cuda.synchronize()
    L, B, P, G = tr.L, tr.B, tr.p, tr.g
    s = _lib.stream_ptr(dev)
    bi = tr.batch_idx.data_ptr()
    da1p = torch.empty(B * 2880, device=dev)
    f3acc = torch.zeros(B * 500, device=dev)
    o = tr._opt_args()
    launches = {
        "conv1_fwd": lambda: L.pto_conv1_fwd(tr.data.data_ptr(), P["conv1.weight"].data_ptr(),
                                             P["conv1.bias"].data_ptr(), tr.a1p.data_ptr(), tr.code1.data_ptr(), B,
                                             bi, s),
        "conv2_fwd": lambda: L.pto_conv2_fwd(tr.a1p.data_ptr(), P["conv2.weight"].data_ptr(),
                                             P["conv2.bias"].data_ptr(), tr.a2p.data_ptr(), tr.code2.data_ptr(), B, s),
        "F12 conv12_fwd": lambda: L.pto_conv12_fwd_lazy_x(
            tr.data.data_ptr(), P["conv1.weight"].data_ptr(), P["conv1.bias"].data_ptr(), P["conv2.weight"].data_ptr(),
            P["conv2.bias"].data_ptr(), tr.a1p.data_ptr(), tr.code1.data_ptr(), tr.a2p.data_ptr(),
            tr.code2.data_ptr(), B, bi, None, None, 0, None, None, 0.0, 0.0, 1.0, 0, tr.xcur.data_ptr(), None, None,
            1, 0, s),
        "F3 fc1_fwd (one workgroup per tile)": lambda: L.pto_linear_fwd(
            tr.a2p.data_ptr(), P["fc1.weight"].data_ptr(), P["fc1.bias"].data_ptr(), tr.h1.data_ptr(), B, 500, 800,
            1, s),
        # the step's form; accumulates into a scratch buffer (timing only)
        "F3 fc1_fwd_split": lambda: L.pto_fc1_fwd_split(tr.a2p.data_ptr(), P["fc1.weight"].data_ptr(),
                                                        f3acc.data_ptr(), B, s),
        "F4dx fc2_ce_dx": lambda: L.pto_fc2_ce_dx(
            tr.h1.data_ptr(), P["fc2.weight"].data_ptr(), P["fc2.bias"].data_ptr(), tr.target.data_ptr(),
            P["fc1.weight"].data_ptr(), tr.loss_rows.data_ptr(), tr.dlogits.data_ptr(), tr.dh1.data_ptr(),
            tr.da2p.data_ptr(), B, 1.0 / B, bi, tr._params[tr._c1:].data_ptr(), tr.grads[tr._c1:].data_ptr(),
            tr.mom[tr._c1:].data_ptr(), tr.numel - tr._c1, None, *o, None, 1, 0, None, None, None, 0, None, None, s),
        "B bwd_all(grads)": lambda: tr._backward(),
        "fc2_ce": lambda: L.pto_fc2_ce(tr.h1.data_ptr(), P["fc2.weight"].data_ptr(), P["fc2.bias"].data_ptr(),
                                       tr.target.data_ptr(), None, tr.loss_rows.data_ptr(), tr.dlogits.data_ptr(),
                                       tr.dh1.data_ptr(), B, 1.0 / B, bi, s),
    }
    for parts, nm, fuse in ((1, "conv2_bwd_wgrad", 0), (2, "conv2_bwd_dgrad", 0), (4, "conv2_bwd_bias", 0),
                            (7, "conv2_bwd_all", 0), (7, "conv2_bwd_all+conv1", 1)):
        launches[nm] = (lambda p=parts, f=fuse: L.pto_conv2_bwd(
            tr.da2p.data_ptr(), tr.code2.data_ptr(), tr.a1p.data_ptr(), P["conv2.weight"].data_ptr(),
            G["conv2.weight"].data_ptr(), G["conv2.bias"].data_ptr(), da1p.data_ptr(), B, p,
            tr.data.data_ptr() if f else None, bi if f else None, tr.code1.data_ptr() if f else None,
            G["conv1.weight"].data_ptr() if f else None, G["conv1.bias"].data_ptr() if f else None, s))
    launches["conv1_bwd"] = lambda: L.pto_conv1_bwd(da1p.data_ptr(), tr.code1.data_ptr(), tr.data.data_ptr(),
                                                    G["conv1.weight"].data_ptr(), G["conv1.bias"].data_ptr(), B, bi, s)
    launches["sgd"] = lambda: tr._sgd_launch()  # ddp-rccl optimizer launch (k_ddp_sgd)
    launches["empty(sgd n=1)"] = None
    tiny = torch.zeros(4, device=dev)
    from pytorch_operator_1_amd.ops.optim import SgdTable

    tt = SgdTable([(tiny, tiny.clone(), None)], dev)
    launches["empty(sgd n=1)"] = lambda: tt.step(None, 0.0, 0.0, 0.0, 1.0, False, zero_grad=False, stream=s)

    names = list(launches)
    times = {n: [] for n in names}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(a.iters):
        for n in names:
            ev[0].record()
            rc = launches[n]()
            ev[1].record()
            if rc not in (None, 0):
                raise RuntimeError(f"{n}: hip error {rc}")
            torch.cuda.synchronize()
            times[n].append(ev[0].elapsed_time(ev[1]) * 1e3)
    out = {}
    for n in names:
        t = sorted(times[n])
        out[n] = {"median_us": round(t[len(t) // 2], 2), "min_us": round(t[0], 2)}
        print(f"{n:20s} median {out[n]['median_us']:8.2f} us   min {out[n]['min_us']:8.2f} us")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
