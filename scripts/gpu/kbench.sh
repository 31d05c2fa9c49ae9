#!/bin/bash
# numerics tests + per-kernel microbench + fused bench
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -50 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python tools/kernel_bench.py --iters 200 --json gpurun_out/kbench.json
timeout -k 10 200 python bench.py --impl fused --steps 3000 --warmup 300 > gpurun_out/fused_bench.json 2> gpurun_out/fused_bench.err
cat gpurun_out/fused_bench.json
