#!/bin/bash
# flash attention numerics first (new kernels), then LLM tests, ops timing, Llama-8B bench
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
: timeout -k 10 300 python -m pytest tests/test_attention_gpu.py -x -q > gpurun_out/pytest_attn.log 2>&1 || { tail -60 gpurun_out/pytest_attn.log; exit 1; }
tail -2 gpurun_out/pytest_attn.log
: timeout -k 10 300 python -m pytest tests/test_llm_gpu.py -x -q > gpurun_out/pytest_llm.log 2>&1 || { tail -60 gpurun_out/pytest_llm.log; exit 1; }
tail -2 gpurun_out/pytest_llm.log
timeout -k 10 300 python tools/llama_ops_bench.py --json gpurun_out/llama_ops.json > gpurun_out/llama_ops.log 2>&1 || { tail -20 gpurun_out/llama_ops.log; exit 1; }
grep -E "sdpa|flash" gpurun_out/llama_ops.log
for b in 2 4; do
timeout -k 10 400 python bench.py --model llama3-8b --batch-size $b --steps 5 --warmup 2 --breakdown > gpurun_out/llama8b_b$b.json 2> gpurun_out/llama8b_b$b.err || { tail -30 gpurun_out/llama8b_b$b.err; exit 1; }
cat gpurun_out/llama8b_b$b.json
done
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/resnet.json 2> gpurun_out/resnet.err || { tail -30 gpurun_out/resnet.err; exit 1; }
cat gpurun_out/resnet.json
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py -x -q > gpurun_out/pytest_mnist.log 2>&1 || { tail -40 gpurun_out/pytest_mnist.log; exit 1; }
tail -2 gpurun_out/pytest_mnist.log
timeout -k 10 200 python tools/kernel_bench.py --iters 200 --json gpurun_out/kbench.json | grep -E "fc|conv12|sgd"
timeout -k 10 200 python bench.py --steps 3000 --warmup 300 > gpurun_out/fused_bench.json 2> gpurun_out/fused_bench.err || { tail -20 gpurun_out/fused_bench.err; exit 1; }
cat gpurun_out/fused_bench.json
