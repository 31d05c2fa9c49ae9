#!/usr/bin/env python3
"""Per-phase timeline of ``k_bwd_all``'s roles: the shipped kernel source
built with its PTO_STAMP marks compiled in (tools/probes/bwd_phases.hip, its
own .so).  Thread 0 of every block stamps the chip-wide 100 MHz clock at
entry, at each phase mark and at exit; the report gives, per role, the mean
entry offset from the launch's first block, mean phase durations and mean
exit, plus the launch span.  Usage: python tools/bwd_phases_probe.py
[--build] [--mask 31]."""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SRC = os.path.join(ROOT, "tools", "probes", "bwd_phases.hip")
SO = os.path.join(ROOT, "tools", "probes", "libbwd_phases.so")
SLOTS = 8
PHASES = {"A": ["staged", "mfma", "atomics done", "counted", "exit"],
          "B": ["staged+dY", "gemm+T", "col2im", "conv1 wgrad", "exit"]}
MARKS = {"A": [0, 1, 2, 3, 4, 7], "B": [0, 1, 3, 4, 5, 7]}


def build():
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                           "-I", os.path.join(ROOT, "pytorch_operator_1_amd", "csrc", "kernels"), "-I", os.path.join(ROOT, "pytorch_operator_1_amd", "csrc", "comm"), "-o", SO, SRC,
                           # mnist_kernels.hip calls pto_ar_timeout_ticks (the exchange roles)
                           os.path.join(ROOT, "pytorch_operator_1_amd", "csrc", "comm", "xgmi_allreduce.hip")])
    print("built", SO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--mask", type=int, nargs="*", default=[31, 8, 4])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--fwd", action="store_true", help="time F12 and F4dx phases instead")
    a = ap.parse_args()
    if a.build:
        build()
        return
    import numpy as np
    import torch

    from pytorch_operator_1_amd.ops import _lib
    from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer

    P_, I_, L_ = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong
    lib = ctypes.CDLL(SO)
    fn = lib.probe_bwd_all
    fn.argtypes = [P_] * 13 + [L_] * 8 + [P_, P_, L_, P_, I_, P_, P_, I_, I_, I_, P_]
    fn.restype = ctypes.c_int
    rd = lib.probe_read_stamps
    rd.argtypes = [P_, I_]
    dev = torch.device("cuda", 0)
    tr = FusedMnistTrainer(dev, batch_size=64, dataset_size=64 * 16, graph="none")
    for _ in range(3):
        tr.step()
    torch.cuda.synchronize()
    if a.fwd:
        return fwd_phases(lib, rd, tr, dev, a.reps)
    counts = dict(C=13, F=17, A=352, B=640, D=400)
    bits = dict(C=1, F=2, A=4, B=8, D=16)
    occ = ctypes.CDLL(SO).probe_bwd_all_occupancy
    occ.restype = ctypes.c_int
    print("resident k_bwd_all blocks per CU (occupancy API):", occ())
    report = {}
    for mask in a.mask:
        spans, per_role = [], {}
        for _ in range(a.reps):
            rc = fn(tr.da2p.data_ptr(), tr.code2.data_ptr(), tr.a1p.data_ptr(), tr.w2f.data_ptr(),
                    tr.xcur.data_ptr(), tr.code1.data_ptr(), tr.dh1.data_ptr(), tr.a2p.data_ptr(), tr.h1.data_ptr(),
                    tr.dlogits.data_ptr(), tr._params.data_ptr(), tr.grads.data_ptr(), tr.mom.data_ptr(),
                    *tr._offs, tr.c2_ctr.data_ptr(), tr.batch_idx.data_ptr(), tr.n_batches, tr.pending.data_ptr(),
                    tr.B, tr.lr_dev.data_ptr(), tr.c1rep.data_ptr(), tr.c1_nrep, tr.c1_stride, mask,
                    _lib.stream_ptr(dev))
            assert rc == 0
            torch.cuda.synchronize()
            nblk = sum(counts[r] for r in counts if mask & bits[r])
            buf = (ctypes.c_ulonglong * (nblk * SLOTS))()
            assert rd(buf, nblk * SLOTS) == 0
            st = np.frombuffer(buf, dtype=np.uint64).reshape(nblk, SLOTS).astype(np.int64)
            t0 = st[:, 0].min()
            rel = (st - t0) * 10.0 / 1000.0  # 100 MHz ticks -> us
            spans.append(float(rel[:, 7].max()))
            i = 0
            for r in ("C", "F", "A", "B", "D"):
                if not mask & bits[r]:
                    continue
                blk = rel[i:i + counts[r]]
                i += counts[r]
                d = per_role.setdefault(r, {"entry": [], "exit": [], "entry_max": [], "exit_max": [], "ph": []})
                d["entry"].append(blk[:, 0].mean())
                d["entry_max"].append(blk[:, 0].max())
                d["exit"].append(blk[:, 7].mean())
                d["exit_max"].append(blk[:, 7].max())
                d.setdefault("entry_hist", []).append(np.histogram(blk[:, 0], bins=[0, 2, 4, 6, 8, 10, 12, 14, 99])[0])
                if r in PHASES:
                    marks = MARKS[r]
                    durs = []
                    for k0, k1 in zip(marks, marks[1:]):
                        ok = (blk[:, k1] > 0) & (blk[:, k0] > 0)
                        durs.append(float((blk[ok, k1] - blk[ok, k0]).mean()) if ok.any() else float("nan"))
                    d["ph"].append(durs)
        med = lambda v: float(np.median(v))
        out = {"span_us": round(med(spans), 2)}
        for r, d in per_role.items():
            o = {"entry_mean": round(med(d["entry"]), 2), "entry_last": round(med(d["entry_max"]), 2),
                 "exit_mean": round(med(d["exit"]), 2), "exit_last": round(med(d["exit_max"]), 2)}
            o["entry_hist_2us"] = [int(v) for v in np.median(np.array(d["entry_hist"]), axis=0)]
            if d["ph"]:
                ph = np.median(np.array(d["ph"]), axis=0)
                o["phases"] = {name: round(float(v), 2) for name, v in zip(PHASES[r], ph)}
            out[r] = o
        report[mask] = out
        print(f"mask {mask}: {json.dumps(out)}")
    print(json.dumps(report))


def fwd_phases(lib, rd, tr, dev, reps):
    """F12 (k_conv12_fwd2_t) and F4dx (k_fc2_ce_dx_mf) with their stamps:
    the probe .so's own copies of the shipped launchers, fused-opt args."""
    import numpy as np
    import torch

    from pytorch_operator_1_amd.ops import _lib

    for name, sig in _lib._SIGS.items():
        if hasattr(lib, name):
            getattr(lib, name).argtypes = sig
            getattr(lib, name).restype = ctypes.c_int
    real = tr.L
    tr.L = lib  # trainer launches through the probe library

    kernels = {"F12": (lambda: tr._forward_part(0), 256, ["staged", "conv1", "conv2+reduce", "exit"], [0, 1, 2, 3, 7]),
               "F3": (lambda: tr._forward_part(1), 256 if getattr(tr, "h1a", None) is not None else 128,
                      ["w0 loads+MFMA", "barrier", "reduce+store"], [0, 1, 2, 7]),
               "F4dx": (lambda: tr._forward_part(2), 201 + 0, ["staged", "Z gemm", "softmax", "dh1", "da2p", "exit"],
                        [0, 1, 2, 3, 4, 5, 7])}
    out = {}
    for k, (fn, nblk, names, marks) in kernels.items():
        ph, spans = [], []
        for _ in range(reps):
            fn()
            torch.cuda.synchronize()
            buf = (ctypes.c_ulonglong * (nblk * SLOTS))()
            assert rd(buf, nblk * SLOTS) == 0
            st = np.frombuffer(buf, dtype=np.uint64).reshape(nblk, SLOTS).astype(np.int64)
            rel = (st - st[:, 0].min()) * 10.0 / 1000.0
            if k == "F4dx":
                rel = rel[:200]  # tile blocks (the commit block has no phases)
            spans.append(float(rel[:, 7].max()))
            ph.append([float((rel[:, k1] - rel[:, k0]).mean()) for k0, k1 in zip(marks, marks[1:])] +
                      [float(rel[:, 0].mean()), float(rel[:, 0].max()), float(rel[:, 7].mean())])
        m = np.median(np.array(ph), axis=0)
        out[k] = {"span_us": round(float(np.median(spans)), 2),
                  "phases": {n: round(float(v), 2) for n, v in zip(names, m)},
                  "entry_mean": round(float(m[-3]), 2), "entry_last": round(float(m[-2]), 2),
                  "exit_mean": round(float(m[-1]), 2)}
        print(k, json.dumps(out[k]))
    tr.L = real
    print(json.dumps(out))


if __name__ == "__main__":
    main()
