#!/bin/bash
# dW1 tile loop with 4 k-groups per memory round (PTO_DW1_NG=4): numerics then A/B bench.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
PTO_DW1_NG=4 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dw1ng.log 2>&1 || { tail -60 gpurun_out/pytest_dw1ng.log; exit 1; }
tail -1 gpurun_out/pytest_dw1ng.log
for rep in 1 2; do
for ng in 8 4; do
PTO_DW1_NG=$ng timeout -k 10 200 python bench.py --steps 4000 --warmup 400 > gpurun_out/dw1_$ng.json 2>/dev/null
echo "ng=$ng $(python -c "import json;d=json.load(open('gpurun_out/dw1_$ng.json'));print(d['value'],d['ms_per_step']*1000)")"
done
done
cd /tmp && PTO_DW1_NG=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_dw1" -o run -- python3 "$R/bench.py" --steps 200 --warmup 20 > "$R/gpurun_out/dw1_prof.log" 2>&1
python3 "$R/tools/rocprof_summary.py" "$R/gpurun_out/prof_dw1" --top 6
