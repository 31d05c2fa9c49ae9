#!/bin/bash
# conv2 dgrad GEMM K tail trimmed to 4 MFMAs (PTO_C2_KTAIL=1): numerics, A/B bench (reversed order) and per-variant kernel profile.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_kt.log 2>&1 || { tail -60 gpurun_out/pytest_kt.log; exit 1; }
tail -1 gpurun_out/pytest_kt.log
for rep in 1 2; do
for ng in 1 0; do
PTO_C2_KTAIL=$ng timeout -k 10 200 python bench.py --steps 4000 --warmup 400 > gpurun_out/kt_$ng.json 2>/dev/null
echo "ng=$ng $(python -c "import json;d=json.load(open('gpurun_out/kt_$ng.json'));print(d['value'],d['ms_per_step']*1000)")"
done
done
cd /tmp
for ng in 0 1; do
PTO_C2_KTAIL=$ng timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_kt_$ng" -o run -- python3 "$R/bench.py" --steps 200 --warmup 20 > "$R/gpurun_out/kt_prof_$ng.log" 2>&1
echo "== ng=$ng"; python3 "$R/tools/rocprof_summary.py" "$R/gpurun_out/prof_kt_$ng" --top 5
done
