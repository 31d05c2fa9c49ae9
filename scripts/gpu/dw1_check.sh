#!/bin/bash
# dW1-in-B1 SGD epilogue: numerics tests, A/B bench, kernel profile.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py tests/test_kernels_gpu.py tests/test_e2e_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_dw1.log 2>&1 || { tail -60 gpurun_out/pytest_dw1.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_dw1.log | tail -2
for r in 1; do
  for v in 0 1; do
    PTO_F4DX=$v timeout -k 10 120 python bench.py --steps 4000 --warmup 300 > gpurun_out/bench_dw1_$v.json 2> gpurun_out/bench_dw1_$v.err
    python -c "import json;d=json.load(open('gpurun_out/bench_dw1_$v.json'));print('f4dx=$v', d['value'], d['ms_per_step'])"
  done
done
R="$GRAFT_REPO_ROOT"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_dw1" -o run -- python3 "$R/bench.py" --steps 200 --warmup 20 > "$R/gpurun_out/prof_dw1.log" 2>&1
python3 "$R/tools/rocprof_summary.py" "$R/gpurun_out/prof_dw1" --top 8
