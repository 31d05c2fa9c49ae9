#!/bin/bash
# ResNet-50 step: rocprofv3 kernel trace, steady-state window (last 3 steps).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
cd /tmp
( while sleep 30; do echo "[prof] $(date +%T) running"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_resnet" -o run -- python3 "$R/bench.py" --model resnet50 --steps 4 --warmup 3 > "$R/gpurun_out/resnet_prof.log" 2>&1 || { tail -30 "$R/gpurun_out/resnet_prof.log"; exit 1; }
grep '^{' "$R/gpurun_out/resnet_prof.log" | cut -c1-200
python3 "$R/tools/rocprof_window.py" "$R/gpurun_out/prof_resnet" --marker sgd --steps 3 --top 40 > "$R/gpurun_out/resnet_window.md"
head -24 "$R/gpurun_out/resnet_window.md"
rm -rf "$R/gpurun_out/prof_resnet"  # large; the window summary is what is kept
