#!/bin/bash
# fused-optimizer schedule: numerics (trainer tests), bench both schedules, kernel trace
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/pytest_fopt.log 2>&1 || { tail -60 gpurun_out/pytest_fopt.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_fopt.log | tail -2
for f in 1 2; do PTO_CONV12=$f timeout -k 10 200 python bench.py --steps 3000 --warmup 300 > gpurun_out/bench_c12_$f.json 2>/dev/null; echo "conv12=$f $(cut -c1-150 gpurun_out/bench_c12_$f.json)"; done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_fopt" -o run -- python3 "$R/bench.py" --steps 200 --warmup 20 > "$R/gpurun_out/prof_fopt.log" 2>&1
python3 "$R/tools/rocprof_summary.py" "$R/gpurun_out/prof_fopt" --top 10
