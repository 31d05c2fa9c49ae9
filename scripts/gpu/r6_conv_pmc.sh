#!/bin/bash
# Round 6: SQ counters of the 3x3 conv kernel vs MIOpen/CK on one shape
# (C=256, 14x14, stride 1), two 8-counter passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
O=gpurun_out/r6pmc
mkdir -p $O
cd /tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM" "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d "/tmp/c3pmc_$i" -o run -- python3 "$R/tools/conv3x3_bench.py" --shapes 256:14:1 --no-dgrad --reps 5 --variants 64:1,64:2 > "$R/$O/pmc_$i.log" 2>&1 || { tail -20 "$R/$O/pmc_$i.log"; exit 1; }
done
python3 "$R/tools/pmc_summary.py" /tmp/c3pmc_1 /tmp/c3pmc_2 --skip 3 > "$R/$O/pmc_summary.txt"
cat "$R/$O/pmc_summary.txt"
