#!/bin/bash
# Per-kernel stats of the MNIST step under rocprofv3 for one or more env
# settings: kstats.sh "PTO_DETERMINISTIC=0" "PTO_DETERMINISTIC=1" ...  Keeps only the
# stats CSVs (the traces are large).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/kstats
cd /tmp
i=0
for setting in "$@"; do
  i=$((i+1))
  d="/tmp/kst_$i"
  rm -rf "$d"
  env $setting true  # validate the assignment syntax
  ( export $setting; timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run -- python3 "$R/bench.py" --steps 200 --warmup 20 --no-latency > "$R/gpurun_out/kstats/run_$i.log" 2>&1 )
  f=$(find "$d" -name "*kernel_stats.csv" | head -1)
  { echo "# $setting"; cat "$f"; } > "$R/gpurun_out/kstats/stats_$i.csv"
  echo "== $setting"; python3 "$R/tools/kstats_table.py" "$f"
  grep -o '"ms_per_step": [0-9.]*' "$R/gpurun_out/kstats/run_$i.log" || true
done
