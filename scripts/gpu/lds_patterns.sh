#!/bin/bash
# SQ_LDS_BANK_CONFLICT per dispatch of the LDS access-pattern probe kernels
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cd /tmp
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES --kernel-trace -d /tmp/ldsp -o run -- python3 "$R/tools/lds_patterns_probe.py" > "$R/gpurun_out/ldsp.log" 2>&1 || { tail -20 "$R/gpurun_out/ldsp.log"; exit 1; }
python3 "$R/tools/pmc_summary.py" /tmp/ldsp --filter p_ --per-dispatch | tee "$R/gpurun_out/ldsp.txt"
