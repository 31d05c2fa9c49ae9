#!/bin/bash
# fused head (fc2+CE) wave reduction by recursive halving + readlane broadcast (PTO_HEAD_HALVING=1): numerics then A/B bench.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
PTO_HEAD_HALVING=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_headhalv.log 2>&1 || { tail -60 gpurun_out/pytest_headhalv.log; exit 1; }
tail -1 gpurun_out/pytest_headhalv.log
for rep in 1 2; do
for ng in 0 1; do
PTO_HEAD_HALVING=$ng timeout -k 10 200 python bench.py --steps 4000 --warmup 400 > gpurun_out/hh_$ng.json 2>/dev/null
echo "ng=$ng $(python -c "import json;d=json.load(open('gpurun_out/hh_$ng.json'));print(d['value'],d['ms_per_step']*1000)")"
done
done
cd /tmp && PTO_HEAD_HALVING=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_hh" -o run -- python3 "$R/bench.py" --steps 200 --warmup 20 > "$R/gpurun_out/hh_prof.log" 2>&1
python3 "$R/tools/rocprof_summary.py" "$R/gpurun_out/prof_hh" --top 6
