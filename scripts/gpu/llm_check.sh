#!/bin/bash
# GPU tests (all) + ResNet-50 / Llama-3 benches + rocprof of the Llama step
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --model llama3-1b --steps 10 --warmup 3 > gpurun_out/llama1b.json 2> gpurun_out/llama1b.err || { tail -30 gpurun_out/llama1b.err; exit 1; }
cat gpurun_out/llama1b.json
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/resnet.json 2> gpurun_out/resnet.err || { tail -30 gpurun_out/resnet.err; exit 1; }
cat gpurun_out/resnet.json
timeout -k 10 500 python bench.py --model llama3-8b --steps 6 --warmup 2 > gpurun_out/llama8b.json 2> gpurun_out/llama8b.err || { tail -30 gpurun_out/llama8b.err; exit 1; }
cat gpurun_out/llama8b.json
