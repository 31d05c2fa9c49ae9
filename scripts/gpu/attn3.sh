#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -m pytest tests/test_attention_gpu.py -x -q > gpurun_out/pytest_attn.log 2>&1 || { tail -60 gpurun_out/pytest_attn.log; exit 1; }
tail -1 gpurun_out/pytest_attn.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_attn" -o run -- python3 "$R/tools/attn_prof.py" > "$R/gpurun_out/attn_trace.log" 2>&1 || { tail -20 "$R/gpurun_out/attn_trace.log"; exit 1; }
python3 "$R/tools/rocprof_summary.py" "$R/gpurun_out/prof_attn" --top 4 | grep attn
