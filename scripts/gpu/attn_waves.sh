#!/bin/bash
# 8-wave forward / dQ attention blocks: numerics (both layouts), op timing, Llama bench.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in 8 4; do
  PTO_ATTN_WAVES=$w timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_attn_$w.log 2>&1 || { tail -40 gpurun_out/pytest_attn_$w.log; exit 1; }
  echo "waves=$w $(tail -1 gpurun_out/pytest_attn_$w.log)"
  PTO_ATTN_WAVES=$w timeout -k 10 300 python tools/llama_ops_bench.py --batch 4 --json gpurun_out/llama_ops_$w.json > gpurun_out/llama_ops_$w.log 2>&1 || { tail -20 gpurun_out/llama_ops_$w.log; exit 1; }
  echo "waves=$w $(grep -E "flash" gpurun_out/llama_ops_$w.log)"
done
PTO_ATTN_WAVES=8 timeout -k 10 300 python -u bench.py --model llama3-8b --steps 5 --warmup 2 > gpurun_out/llama_w8.json 2>/dev/null
cut -c1-170 gpurun_out/llama_w8.json
