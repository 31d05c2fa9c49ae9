#!/usr/bin/env python3
"""Which roles of ``k_bwd_all`` set its time: the launch with whole block
ranges left out (tools/probes/bwd_roles.hip, its own .so; the shipped
kernel is unchanged).  Each variant: a HIP graph of 40 launches, replayed,
median us per launch.  Usage: python tools/bwd_roles_probe.py [--build]
(--build compiles the probe .so, on the CPU host, before the GPU run)."""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SRC = os.path.join(ROOT, "tools", "probes", "bwd_roles.hip")
SO = os.path.join(ROOT, "tools", "probes", "libbwd_roles.so")
ROLES = {1: "C conv2-bias", 2: "F fc2/bias", 4: "A conv2-wgrad", 8: "B dgrad+conv1-wgrad", 16: "D dW1", 32: "-c1 (B without its conv1 wgrad)"}


def so_path(chunk, dtpw=None, order=None):
    p = SO if chunk is None else SO.replace(".so", f"_c{chunk}.so")
    p = p if dtpw is None else p.replace(".so", f"_d{dtpw}.so")
    return p if order is None else p.replace(".so", f"_o{order}.so")


def build(chunk=None, dtpw=None, order=None):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-I", os.path.join(ROOT, "pytorch_operator_1_amd", "csrc", "kernels"), "-I", os.path.join(ROOT, "pytorch_operator_1_amd", "csrc", "comm"), "-o", so_path(chunk, dtpw, order), SRC,
           # mnist_kernels.hip calls pto_ar_timeout_ticks (the exchange roles)
           os.path.join(ROOT, "pytorch_operator_1_amd", "csrc", "comm", "xgmi_allreduce.hip")]
    if chunk is not None:
        cmd.insert(1, f"-DPTO_BWD_WCHUNK={chunk}")
    if dtpw is not None:  # the serial tiles-per-wave form (PTO_BWD_DPAIR is then off)
        cmd.insert(1, f"-DPTO_BWD_DTPW={dtpw}")
    if order is not None:
        cmd.insert(1, f"-DPTO_BWD_ORDER={order}")
    subprocess.check_call(cmd)
    print("built", so_path(chunk, dtpw, order))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--chunk", type=int, nargs="*", default=None,
                    help="conv2-wgrad samples per block to sweep (each its own probe build)")
    ap.add_argument("--dtpw", type=int, nargs="*", default=None,
                    help="dW1 tiles per wave of the D blocks to sweep (each its own probe build)")
    ap.add_argument("--dpair", type=int, nargs="*", default=None,
                    help="PTO_BWD_DPAIR values (0: one dW1 tile per wave, 1: a pair side by side) to "
                         "compare, interleaved (a host switch of the same build)")
    ap.add_argument("--order", type=int, nargs="*", default=None,
                    help="k_bwd_all role orders (mnist_kernels.hip bwd_order) to sweep (each its own probe build)")
    ap.add_argument("--pmc-mask", type=int, default=None,
                    help="no timing: 30 eager launches of this role mask, for a rocprofv3 --pmc run "
                         "(pmc_summary.py --skip 3 drops the trainer's own 3 warm-up dispatches)")
    a = ap.parse_args()
    if a.build:
        for c in (a.chunk or [None]):
            for d in (a.dtpw or [None]):
                for o in (a.order or [None]):
                    build(c, d, o)
        return
    if a.dpair:
        for rep in range(2):  # interleaved A/B
            for pr in a.dpair:
                print(f"== dW1 tile pairs {pr} (pass {rep})")
                run_one(SO, a.reps, masks=[31, 16, 31 & ~16], dpair=pr)
        return
    if a.order:
        for o in a.order:
            print(f"== role order {o}")
            run_one(so_path(None, None, o), a.reps, masks=[31])
        return
    if a.dtpw:
        for d in a.dtpw:
            print(f"== dW1 tiles per wave {d}")
            run_one(so_path(None, d), a.reps, masks=[31, 16, 31 & ~16])
        return
    if a.chunk:
        for c in a.chunk:
            print(f"== wgrad chunk {c}")
            run_one(so_path(c), a.reps, masks=[31, 4, 8])
        return
    run_one(SO, a.reps, pmc_mask=a.pmc_mask)


def run_one(so, reps, masks=None, pmc_mask=None, dpair=None):
    import torch

    from pytorch_operator_1_amd.ops import _lib
    from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer

    P_, I_, L_ = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong
    if dpair is not None:  # read once per process by bwd_dpair(): one CDLL copy per setting
        os.environ["PTO_BWD_DPAIR"] = str(dpair)
        so_copy = so.replace(".so", f"_dp{dpair}.so")
        if not os.path.exists(so_copy):
            import shutil
            shutil.copy(so, so_copy)
        so = so_copy
    lib = ctypes.CDLL(so)
    fn = lib.probe_bwd_all
    fn.argtypes = [P_] * 13 + [L_] * 8 + [P_, P_, L_, P_, I_, P_, P_, I_, I_, I_, P_]
    fn.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    tr = FusedMnistTrainer(dev, batch_size=64, dataset_size=64 * 16, graph="none")
    for _ in range(3):
        tr.step()
    torch.cuda.synchronize()

    def launch(mask):
        rc = fn(tr.da2p.data_ptr(), tr.code2.data_ptr(), tr.a1p.data_ptr(), tr.w2f.data_ptr(), tr.xcur.data_ptr(),
                tr.code1.data_ptr(), tr.dh1.data_ptr(), tr.a2p.data_ptr(), tr.h1.data_ptr(), tr.dlogits.data_ptr(),
                tr._params.data_ptr(), tr.grads.data_ptr(), tr.mom.data_ptr(), *tr._offs, tr.c2_ctr.data_ptr(),
                tr.batch_idx.data_ptr(), tr.n_batches, tr.pending.data_ptr(), tr.B, tr.lr_dev.data_ptr(),
                tr.c1rep.data_ptr(), tr.c1_nrep, tr.c1_stride, mask, _lib.stream_ptr(dev))
        assert rc == 0, rc

    if pmc_mask is not None:
        for _ in range(30):
            launch(pmc_mask)
        torch.cuda.synchronize()
        return
    masks = masks or [31, 1 | 2, 4, 8, 16, 31 & ~4, 31 & ~8, 31 & ~16, 4 | 8]
    graphs = {}
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        for mk in masks:
            launch(mk)
    torch.cuda.synchronize()
    for mk in masks:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(40):
                launch(mk)
        graphs[mk] = g
    res = {mk: [] for mk in masks}
    for _ in range(reps):
        for mk in masks:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            graphs[mk].replay()
            e1.record()
            e1.synchronize()
            res[mk].append(e0.elapsed_time(e1) * 1000 / 40)
    out = {}
    for mk in masks:
        v = sorted(res[mk])[len(res[mk]) // 2]
        name = "+".join(ROLES[b].split()[0] for b in ROLES if mk & b) or "empty grid (noop)"
        out[name] = round(v, 2)
        print(f"{name:>24s}  {v:7.2f} us/launch")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
