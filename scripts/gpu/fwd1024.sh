#!/bin/bash
# 1024-thread fused forward (PTO_FWD_THREADS=1024): numerics, reversed-order A/B, then the round check with it on.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
PTO_FWD_THREADS=1024 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_f1k.log 2>&1 || { tail -60 gpurun_out/pytest_f1k.log; exit 1; }
tail -1 gpurun_out/pytest_f1k.log
for rep in 1 2; do
for ng in 1024 512; do
PTO_FWD_THREADS=$ng timeout -k 10 200 python bench.py --steps 4000 --warmup 400 > gpurun_out/f1k_$ng.json 2>/dev/null
echo "ng=$ng $(python -c "import json;d=json.load(open('gpurun_out/f1k_$ng.json'));print(d['value'],d['ms_per_step']*1000)")"
done
done
export PTO_FWD_THREADS=1024
bash scripts/gpu/round_check.sh
