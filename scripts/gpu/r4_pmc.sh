#!/bin/bash
# Round-4 SQ counters: the N=1 step (scripts/gpu/r2_pmc.sh r4) and the
# overlapped ddp-xgmi step at world 1 (F12 with the fc all-reduce role, the
# one-shot conv exchange, the closing role launch).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
bash scripts/gpu/r2_pmc.sh r4
cd /tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d "/tmp/ddp_pmc_$i" -o run -- python3 "$R/tools/ddp_step_bench.py" --only xgmi --steps 40 --warmup 8 > "$R/gpurun_out/ddp_pmc_$i.log" 2>&1 || { tail -20 "$R/gpurun_out/ddp_pmc_$i.log"; exit 1; }
done
python3 "$R/tools/pmc_summary.py" /tmp/ddp_pmc_1 /tmp/ddp_pmc_2 --filter k_ --skip 3 > "$R/gpurun_out/ddp_pmc_summary.txt"
cat "$R/gpurun_out/ddp_pmc_summary.txt"
