#!/bin/bash
# ResNet-50 step (owned 3x3 convs) under a kernel trace: per-kernel window
# summary of the last 2 steps.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
O=$R/gpurun_out/r6_rwin
mkdir -p $O
cd /tmp
( while sleep 30; do echo "[prof] $(date +%T) running"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/prof_rw -o run -- python3 "$R/bench.py" --model resnet50 --steps 3 --warmup 3 --no-latency > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
grep '^{' $O/prof.log | cut -c1-200
python3 "$R/tools/rocprof_window.py" /tmp/prof_rw --marker sgd --steps 2 --top 60 > $O/window.md
head -75 $O/window.md
