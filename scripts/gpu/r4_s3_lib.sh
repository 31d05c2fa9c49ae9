#!/bin/bash
# first-launch cost of libpto_hip.so's kernels in a fresh GPU process
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/st
cat > gpurun_out/st/lib_probe.py <<'PY'
import json, os, sys, time
sys.path.insert(0, os.getcwd())
import torch
out = {}
t = time.time(); torch.zeros(1, device="cuda"); torch.cuda.synchronize(); out["torch_first_launch_s"] = round(time.time() - t, 4)
from pytorch_operator_1_amd.ops import _lib
t = time.time(); L = _lib.lib(); out["dlopen_s"] = round(time.time() - t, 4)
a = torch.zeros(64, device="cuda"); b = torch.zeros(64, device="cuda"); o = torch.zeros(4096, device="cuda")
s = _lib.stream_ptr(torch.device("cuda", 0))
for k in range(3):
    torch.cuda.synchronize()
    t = time.time(); _lib.check(L.pto_lane_ops_selftest(a.data_ptr(), b.data_ptr(), o.data_ptr(), s), "x"); tl = time.time() - t
    torch.cuda.synchronize(); out[f"selftest{k}_launch_s"] = round(tl, 4); out[f"selftest{k}_total_s"] = round(time.time() - t, 4)
x = torch.empty((60000, 1, 28, 28), device="cuda"); y = torch.empty(60000, device="cuda", dtype=torch.int64)
for k in range(2):
    torch.cuda.synchronize()
    t = time.time(); _lib.check(L.pto_synth_mnist(x.data_ptr(), y.data_ptr(), 60000, 123, s), "s"); torch.cuda.synchronize()
    out[f"synth{k}_s"] = round(time.time() - t, 4)
print(json.dumps(out))
PY
timeout -k 10 120 python gpurun_out/st/lib_probe.py
