#!/bin/bash
# 16-wave fc1 forward: numerics (linear + fused-step graph tests) then A/B bench and kernel times.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
PTO_LINEAR_WAVES=16 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fc16.log 2>&1 || { tail -60 gpurun_out/pytest_fc16.log; exit 1; }
tail -1 gpurun_out/pytest_fc16.log
for rep in 1 2; do
for wv in 8 16; do
PTO_LINEAR_WAVES=$wv timeout -k 10 200 python bench.py --steps 4000 --warmup 400 > gpurun_out/fc_$wv.json 2>/dev/null
echo "waves=$wv $(python -c "import json;d=json.load(open('gpurun_out/fc_$wv.json'));print(d['value'],d['ms_per_step']*1000)")"
done
done
cd /tmp && PTO_LINEAR_WAVES=16 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_fc16" -o run -- python3 "$R/bench.py" --steps 200 --warmup 20 > "$R/gpurun_out/fc16_prof.log" 2>&1
python3 "$R/tools/rocprof_summary.py" "$R/gpurun_out/prof_fc16" --top 6
