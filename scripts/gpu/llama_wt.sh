#!/bin/bash
# W^T dgrad: numerics tests, then the Llama-3-8B bench with and without it.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_llm_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_llm.log 2>&1 || { tail -60 gpurun_out/pytest_llm.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_llm.log | tail -1
for wt in 1; do
  PTO_WT=$wt timeout -k 10 300 python -u bench.py --model llama3-8b --steps 5 --warmup 2 --breakdown > gpurun_out/llama_wt$wt.json 2> gpurun_out/llama_wt$wt.err || { tail -20 gpurun_out/llama_wt$wt.err; exit 1; }
  echo "wt=$wt $(cut -c1-160 gpurun_out/llama_wt$wt.json) $(grep 'phase ms' gpurun_out/llama_wt$wt.err)"
done
