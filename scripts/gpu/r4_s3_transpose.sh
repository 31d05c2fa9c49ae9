#!/bin/bash
# register-transpose kernel: exactness tests, shape sweep vs torch, then the
# Llama-3-8B step (20 timed steps) on the new kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/tp
timeout -k 10 300 python -u -m pytest tests/test_llm_gpu.py tests/test_linear_tw.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tp/pytest.log 2>&1 || { tail -30 gpurun_out/tp/pytest.log; exit 1; }
tail -2 gpurun_out/tp/pytest.log
timeout -k 10 200 python tools/transpose_bench.py > gpurun_out/tp/tp2.jsonl 2> gpurun_out/tp/tp2.err || { tail -20 gpurun_out/tp/tp2.err; exit 1; }
cat gpurun_out/tp/tp2.jsonl
( while sleep 20; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -u bench.py --model llama3-8b --steps 20 --warmup 3 > gpurun_out/tp/llama.json 2> gpurun_out/tp/llama.err || { tail -20 gpurun_out/tp/llama.err; exit 1; }
cat gpurun_out/tp/llama.json
