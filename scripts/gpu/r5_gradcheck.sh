#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5r
mkdir -p $O
for cfg in "256 224" "8 64"; do
PYTHONPATH=. timeout -k 10 300 python tools/probes/resnet_grad_check.py $cfg > $O/gradcheck.txt 2>&1 || { tail -20 $O/gradcheck.txt; exit 1; }
echo "== $cfg"; grep -v amdgpu.ids $O/gradcheck.txt
done
