#!/bin/bash
# SQ counters + kernel trace of the attention backward with the role-split dK/dV kernel.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cd /tmp
export PTO_ATTN_DKDV_SPLIT=1
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/attn_trace_split" -o run -- python3 "$R/tools/attn_prof.py" > "$R/gpurun_out/attn_trace_split.log" 2>&1 || { tail -20 "$R/gpurun_out/attn_trace_split.log"; exit 1; }
python3 "$R/tools/rocprof_summary.py" "$R/gpurun_out/attn_trace_split" --top 5
ITERS=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-trace -d "$R/gpurun_out/attn_pmc_split" -o run -- python3 "$R/tools/attn_prof.py" > "$R/gpurun_out/attn_pmc_split.log" 2>&1 || { tail -20 "$R/gpurun_out/attn_pmc_split.log"; exit 1; }
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/attn_pmc_split" --filter dkdv
