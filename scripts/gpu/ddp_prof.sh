#!/bin/bash
# DDP-schedule step at world size 1 (grads-only backward + RCCL all-reduce of
# a 1-rank group + SGD launch) under rocprofv3: per-kernel stats
# (gpurun_out/ddp_kstats.txt), next to the one-process step's.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cd /tmp
for s in ddp xgmi single; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kst_$s -o run -- python3 "$R/tools/ddp_step_bench.py" --steps 400 --warmup 40 --only $s > "$R/gpurun_out/ddp_prof_$s.log" 2>&1
  f=$(find /tmp/kst_$s -name "*kernel_stats.csv" | head -1)
  echo "== $s $(grep -o '{.*}' $R/gpurun_out/ddp_prof_$s.log | tail -1)"
  python3 "$R/tools/kstats_table.py" "$f" --top 8 | tee "$R/gpurun_out/ddp_kstats_$s.txt"
done
