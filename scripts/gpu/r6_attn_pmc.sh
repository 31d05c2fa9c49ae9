#!/bin/bash
# SQ counters of the attention backward kernels (dK/dV 8-wave PC = 1 and
# 12-wave P3 = 2) at the Llama-3-8B shape, three passes each, plus a kernel
# trace with per-kernel times.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
O=gpurun_out/r6_attn_pmc
mkdir -p $O
cd /tmp
for v in 1 2; do
  PTO_ATTN_DKDV_PC=$v ITERS=3 timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d /tmp/ak_$v -o run -- python3 "$R/tools/attn_ab.py" > "$R/$O/kt_$v.log" 2>&1 || { tail -20 "$R/$O/kt_$v.log"; exit 1; }
  find /tmp/ak_$v -name "*kernel_stats.csv" -exec cp {} "$R/$O/kstats_$v.csv" \;
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM" "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD" "SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    PTO_ATTN_DKDV_PC=$v ITERS=2 timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d "/tmp/apmc_${v}_$i" -o run -- python3 "$R/tools/attn_ab.py" > "$R/$O/pmc_${v}_$i.log" 2>&1 || { tail -20 "$R/$O/pmc_${v}_$i.log"; exit 1; }
  done
  python3 "$R/tools/pmc_summary.py" /tmp/apmc_${v}_1 /tmp/apmc_${v}_2 /tmp/apmc_${v}_3 --filter attn --skip 2 > "$R/$O/pmc_summary_$v.txt"
  echo "== dkdv_pc=$v"; cat "$R/$O/pmc_summary_$v.txt"
  grep -i attn "$R/$O/kstats_$v.csv" | cut -d, -f1-8
done
