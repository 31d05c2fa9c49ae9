#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
cd /tmp
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/counters.txt" 2>&1 || true
grep -oE "^\s*(SQ_[A-Z_0-9]+|[A-Za-z]+Util[A-Za-z]*|[A-Za-z]*Busy[A-Za-z]*|LDS[A-Za-z]*|TCP_[A-Z_]+|GRBM_[A-Z_]+)" "$R/gpurun_out/counters.txt" | sort -u | tr '\n' ' ' | head -c 6000; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_attn" -o run -- python3 "$R/tools/attn_prof.py" > "$R/gpurun_out/attn_trace.log" 2>&1 || { tail -20 "$R/gpurun_out/attn_trace.log"; exit 1; }
python3 "$R/tools/rocprof_summary.py" "$R/gpurun_out/prof_attn" --top 8 | head -16
