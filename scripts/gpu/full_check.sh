#!/bin/bash
# GPU round: all gpu tests (kernels, DDP, whole stack) + bench + rocprof.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -s > gpurun_out/pytest_gpu.log 2>&1 || { tail -80 gpurun_out/pytest_gpu.log; exit 1; }
grep -E "passed|failed|submit ->" gpurun_out/pytest_gpu.log | tail -5
timeout -k 10 200 python tools/kernel_bench.py --iters 200 --json gpurun_out/kbench.json
timeout -k 10 200 python bench.py --steps 3000 --warmup 300 > gpurun_out/fused_bench.json 2> gpurun_out/fused_bench.err
cat gpurun_out/fused_bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_fused" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 200 --warmup 20 > "$GRAFT_REPO_ROOT/gpurun_out/fused_prof.log" 2>&1
echo done
