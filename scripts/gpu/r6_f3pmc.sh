#!/bin/bash
# SQ counters of the fc1 forward (and the other three launches) with the
# split-K fc1 (default) and with one 16-wave workgroup per tile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
O=gpurun_out/r6_f3pmc
mkdir -p $O
cd /tmp
for v in 1 0; do
  timeout -s KILL 120 env PTO_FC1_SPLIT=$v true || exit 1
  export PTO_FC1_SPLIT=$v
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU --kernel-trace -d "/tmp/f3_pmc_$v" -o run -- python3 "$R/bench.py" --steps 20 --warmup 4 --no-latency > "$R/$O/pmc_$v.log" 2>&1 || { tail -20 "$R/$O/pmc_$v.log"; exit 1; }
  python3 "$R/tools/pmc_summary.py" /tmp/f3_pmc_$v --filter k_ --skip 3 > "$R/$O/pmc_summary_$v.txt"
  echo "== PTO_FC1_SPLIT=$v"; cat "$R/$O/pmc_summary_$v.txt"
done
