#!/bin/bash
# rocprofv3 kernel trace of the Llama-3-8B step (kernel sequence of one step)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_llama_wt" -o run -- python3 "$R/bench.py" --model llama3-8b --steps 2 --warmup 1 > "$R/gpurun_out/llama_wt_prof.log" 2>&1 || { tail -30 "$R/gpurun_out/llama_wt_prof.log"; exit 1; }
python3 "$R/tools/rocprof_summary.py" "$R/gpurun_out/prof_llama_wt" --steps 3 --top 14
