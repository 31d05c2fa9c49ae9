#!/bin/bash
# GPU round-trip: kernel numerics tests -> fused bench -> rocprof kernel trace.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -50 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 200 python bench.py --impl fused --steps 2000 --warmup 200 > gpurun_out/fused_bench.json 2> gpurun_out/fused_bench.err
cat gpurun_out/fused_bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_fused" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --impl fused --steps 200 --warmup 20 > "$GRAFT_REPO_ROOT/gpurun_out/fused_prof.log" 2>&1
echo done
