#!/bin/bash
# rocprofv3 kernel-trace profiles of the Llama-3-8B and ResNet-50 steps.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
export PYTHONPATH="$R${PYTHONPATH:+:$PYTHONPATH}"
cd /tmp
timeout -k 10 300 python3 "$R/tools/llama_ops_bench.py" --json "$R/gpurun_out/llama_ops.json" > "$R/gpurun_out/llama_ops.log" 2>&1 || { tail -20 "$R/gpurun_out/llama_ops.log"; exit 1; }
cat "$R/gpurun_out/llama_ops.log"
timeout -k 10 300 python3 "$R/bench.py" --model llama3-8b --steps 4 --warmup 2 --breakdown > "$R/gpurun_out/llama8b_bd.json" 2> "$R/gpurun_out/llama8b_bd.err" || { tail -20 "$R/gpurun_out/llama8b_bd.err"; exit 1; }
grep "phase ms" "$R/gpurun_out/llama8b_bd.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_llama8b" -o run -- python3 "$R/bench.py" --model llama3-8b --steps 3 --warmup 1 > "$R/gpurun_out/llama8b_prof.log" 2>&1 || { tail -30 "$R/gpurun_out/llama8b_prof.log"; exit 1; }
python3 "$R/tools/rocprof_summary.py" "$R/gpurun_out/prof_llama8b" --steps 4 --top 30 > "$R/gpurun_out/llama8b_summary.md"
head -45 "$R/gpurun_out/llama8b_summary.md"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_resnet" -o run -- python3 "$R/bench.py" --model resnet50 --steps 5 --warmup 2 > "$R/gpurun_out/resnet_prof.log" 2>&1 || { tail -30 "$R/gpurun_out/resnet_prof.log"; exit 1; }
python3 "$R/tools/rocprof_summary.py" "$R/gpurun_out/prof_resnet" --steps 7 --top 30 > "$R/gpurun_out/resnet_summary.md"
head -45 "$R/gpurun_out/resnet_summary.md"
