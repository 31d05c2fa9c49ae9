#!/bin/bash
# Llama-3-8B step: phase breakdown + rocprofv3 kernel trace summary.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
cd /tmp
timeout -k 10 300 python3 "$R/bench.py" --model llama3-8b --steps 4 --warmup 2 --breakdown > "$R/gpurun_out/llama8b_bd.json" 2> "$R/gpurun_out/llama8b_bd.err" || { tail -20 "$R/gpurun_out/llama8b_bd.err"; exit 1; }
grep "phase ms" "$R/gpurun_out/llama8b_bd.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_llama8b" -o run -- python3 "$R/bench.py" --model llama3-8b --steps 3 --warmup 1 > "$R/gpurun_out/llama8b_prof.log" 2>&1 || { tail -30 "$R/gpurun_out/llama8b_prof.log"; exit 1; }
python3 "$R/tools/rocprof_summary.py" "$R/gpurun_out/prof_llama8b" --steps 4 --top 40 > "$R/gpurun_out/llama8b_summary.md"
head -50 "$R/gpurun_out/llama8b_summary.md"
