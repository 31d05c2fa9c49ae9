#!/bin/bash
# conv1 weight-grad blocks with the recursive-halving wave reduction (PTO_CONV1_HALVING=1): numerics then A/B bench.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
PTO_CONV1_HALVING=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_c1halv.log 2>&1 || { tail -60 gpurun_out/pytest_c1halv.log; exit 1; }
tail -1 gpurun_out/pytest_c1halv.log
for rep in 1 2; do
for ng in 0 1; do
PTO_CONV1_HALVING=$ng timeout -k 10 200 python bench.py --steps 4000 --warmup 400 > gpurun_out/c1h_$ng.json 2>/dev/null
echo "ng=$ng $(python -c "import json;d=json.load(open('gpurun_out/c1h_$ng.json'));print(d['value'],d['ms_per_step']*1000)")"
done
done
cd /tmp && PTO_CONV1_HALVING=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c1h" -o run -- python3 "$R/bench.py" --steps 200 --warmup 20 > "$R/gpurun_out/c1h_prof.log" 2>&1
python3 "$R/tools/rocprof_summary.py" "$R/gpurun_out/prof_c1h" --top 6
