#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_attention_gpu.py -x -q > gpurun_out/pytest_attn.log 2>&1 || { tail -60 gpurun_out/pytest_attn.log; exit 1; }
tail -1 gpurun_out/pytest_attn.log
timeout -k 10 300 python tools/llama_ops_bench.py --json gpurun_out/llama_ops.json > gpurun_out/llama_ops.log 2>&1 || { tail -20 gpurun_out/llama_ops.log; exit 1; }
grep -E "sdpa_gqa|flash" gpurun_out/llama_ops.log
timeout -k 10 400 python bench.py --model llama3-8b --batch-size 4 --steps 5 --warmup 2 --breakdown > gpurun_out/llama8b_b4.json 2> gpurun_out/llama8b_b4.err || { tail -30 gpurun_out/llama8b_b4.err; exit 1; }
cat gpurun_out/llama8b_b4.json
for f in 0 1; do PTO_FUSE_FC=$f timeout -k 10 200 python bench.py --steps 3000 --warmup 300 > gpurun_out/fused_bench_$f.json 2>/dev/null; echo "fuse_fc=$f $(cut -c1-120 gpurun_out/fused_bench_$f.json)"; done
