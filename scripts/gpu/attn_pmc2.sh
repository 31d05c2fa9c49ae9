#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
cd /tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY" "SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  ITERS=1 timeout -k 10 200 rocprofv3 --pmc $grp --kernel-trace -d "$R/gpurun_out/pmc_attn_$i" -o run -- python3 "$R/tools/attn_prof.py" > "$R/gpurun_out/pmc_$i.log" 2>&1 || { tail -20 "$R/gpurun_out/pmc_$i.log"; exit 1; }
done
ls -R "$R/gpurun_out/pmc_attn_1" | head
