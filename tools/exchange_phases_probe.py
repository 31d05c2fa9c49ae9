#!/usr/bin/env python3
"""Per-phase timeline of the overlapped multi-GPU step's F12 launch (the
previous step's conv + fc exchange as roles, then the convolutions), at
world size 1 (force_ddp, xGMI, eager launches): the shipped kernel source
built with its PTO_STAMP marks (tools/probes/exchange_phases.hip, its own
.so) replaces pto_conv12_fwd_ar.  Reports mean offsets from the launch's
first block entry, per role.  Usage: python tools/exchange_phases_probe.py
[--build] [--steps 40]."""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SRC = os.path.join(ROOT, "tools", "probes", "exchange_phases.hip")
SO = os.path.join(ROOT, "tools", "probes", "libexchange_phases.so")
SLOTS = 8


def build():
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                           "-I", os.path.join(ROOT, "pytorch_operator_1_amd", "csrc", "kernels"), "-I",
                           os.path.join(ROOT, "pytorch_operator_1_amd", "csrc", "comm"), "-o", SO, SRC])
    print("built", SO)


class _LibProxy:
    def __init__(self, real, probe):
        self._real, self._probe = real, probe

    def __getattr__(self, name):
        if name == "pto_conv12_fwd_ar":
            return self._probe.pto_conv12_fwd_ar
        return getattr(self._real, name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--steps", type=int, default=40)
    a = ap.parse_args()
    if a.build:
        build()
        return
    import numpy as np
    import torch

    from pytorch_operator_1_amd.ops import _lib
    from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer

    probe = ctypes.CDLL(SO)
    probe.pto_conv12_fwd_ar.argtypes = _lib._SIGS["pto_conv12_fwd_ar"]
    probe.pto_conv12_fwd_ar.restype = ctypes.c_int
    probe.probe_read_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    tr = FusedMnistTrainer(dev, batch_size=64, dataset_size=64 * 16, graph="none", force_ddp=True, comm="xgmi")
    assert tr._inline
    tr.L = _LibProxy(tr.L, probe)
    from pytorch_operator_1_amd.ops import _lib as L_

    cnb = L_.lib().pto_ar_oneshot_role_blocks(tr.numel - tr._split, 1)
    fnb = None
    rows = []
    buf = np.zeros(4096 * SLOTS, dtype=np.uint64)
    for it in range(a.steps):
        tr._forward(owed=True)  # F12 with both roles (the previous step's exchange), F3, F4dx
        torch.cuda.synchronize()
        assert probe.probe_read_stamps(buf.ctypes.data, buf.size) == 0
        tr._backward()
        torch.cuda.synchronize()
        if it < 5:
            continue
        st = buf.reshape(4096, SLOTS).astype(np.int64)
        nb = int((st[:, 0] > 0).sum())
        t0 = st[:nb, 0][st[:nb, 0] > 0].min()
        rows.append((st[:nb] - t0, nb))
    nb = rows[0][1]
    conv_blocks = 64 * 4
    fnb = nb - cnb - conv_blocks
    out = {"blocks": {"conv_role": cnb, "fc_role": fnb, "conv": conv_blocks}}
    ms = np.mean([r[0] for r in rows], axis=0) / 100.0  # ticks (10 ns) -> us
    cr = ms[:cnb]
    out["conv_role_us"] = {"entry": round(float(cr[:, 0].mean()), 2), "barrier0": round(float(cr[:, 1].mean()), 2),
                           "sgd_issued": round(float(cr[:, 2].mean()), 2), "published": round(float(cr[:, 3].mean()), 2),
                           "published_last": round(float(cr[:, 3].max()), 2),
                           "barrier1": round(float(cr[:, 4].mean()), 2), "exit": round(float(cr[:, 7].mean()), 2)}
    fr = ms[cnb:cnb + fnb]
    out["fc_role_us"] = {"entry": round(float(fr[:, 0].mean()), 2), "exit_mean": round(float(fr[:, 7].mean()), 2),
                         "exit_last": round(float(fr[:, 7].max()), 2)}
    cb = ms[cnb + fnb:]
    out["conv_blocks_us"] = {"entry": round(float(cb[:, 0].mean()), 2), "wait_over": round(float(cb[:, 5].mean()), 2),
                             "staged": round(float(cb[:, 1].mean()), 2), "conv1": round(float(cb[:, 2].mean()), 2),
                             "conv2": round(float(cb[:, 3].mean()), 2), "exit_mean": round(float(cb[:, 7].mean()), 2),
                             "exit_last": round(float(cb[:, 7].max()), 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
