#!/bin/bash
# conv1 per-SIMD task slots A/B (numerics with slots on, reversed-order bench pairs), then the round check on defaults.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
PTO_CONV1_SLOTS=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sl.log 2>&1 || { tail -60 gpurun_out/pytest_sl.log; exit 1; }
tail -1 gpurun_out/pytest_sl.log
for rep in 1 2; do
for ng in 1 0; do
PTO_CONV1_SLOTS=$ng timeout -k 10 200 python bench.py --steps 4000 --warmup 400 > gpurun_out/sl_$ng.json 2>/dev/null
echo "ng=$ng $(python -c "import json;d=json.load(open('gpurun_out/sl_$ng.json'));print(d['value'],d['ms_per_step']*1000)")"
done
done
bash scripts/gpu/round_check.sh
