#!/bin/bash
# LLM/ResNet tests + benches (batch sweep for Llama-8B memory sizing)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_llm_gpu.py -x -q > gpurun_out/pytest_llm.log 2>&1 || { tail -60 gpurun_out/pytest_llm.log; exit 1; }
tail -2 gpurun_out/pytest_llm.log
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/resnet.json 2> gpurun_out/resnet.err || { tail -30 gpurun_out/resnet.err; exit 1; }
cat gpurun_out/resnet.json
for b in 2 4; do
timeout -k 10 400 python bench.py --model llama3-8b --batch-size $b --steps 5 --warmup 2 --breakdown > gpurun_out/llama8b_b$b.json 2> gpurun_out/llama8b_b$b.err || { tail -30 gpurun_out/llama8b_b$b.err; exit 1; }
cat gpurun_out/llama8b_b$b.json
done
