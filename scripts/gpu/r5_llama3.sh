#!/bin/bash
# Llama-3-8B kernel window (last 2 of 3 timed steps).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
O=$R/gpurun_out/r5l3
mkdir -p $O
cd /tmp
( while sleep 30; do echo "[prof] $(date +%T) running"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 rocprofv3 --kernel-trace -d /tmp/prof_ll3 -o run -- python3 "$R/bench.py" --model llama3-8b --steps 3 --warmup 2 --no-latency > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
python3 "$R/tools/rocprof_window.py" /tmp/prof_ll3 --marker adamw --steps 2 --top 20 > $O/window.md
head -24 $O/window.md | cut -c1-150
