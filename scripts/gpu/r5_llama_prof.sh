#!/bin/bash
# Llama-3-8B step: kernel trace, steady-state window (last 2 steps).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
O=$R/gpurun_out/r5l2
mkdir -p $O
cd /tmp
( while sleep 30; do echo "[prof] $(date +%T) running"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 rocprofv3 --kernel-trace -d /tmp/prof_ll -o run -- python3 "$R/bench.py" --model llama3-8b --steps 3 --warmup 2 --no-latency > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
grep '^{' $O/prof.log | cut -c1-200
python3 "$R/tools/rocprof_window.py" /tmp/prof_ll --marker adamw --steps 2 --top 40 > $O/window.md
head -45 $O/window.md
