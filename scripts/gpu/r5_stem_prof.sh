#!/bin/bash
# ResNet-50 kernel windows with and without the MFMA stem kernel.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
O=$R/gpurun_out/r5st
mkdir -p $O
cd /tmp
( while sleep 30; do echo "[prof] $(date +%T) running"; done ) &
HB=$!
trap "kill $HB" EXIT
for v in 1 0; do
PTO_STEM=$v timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/prof_st$v -o run -- python3 "$R/bench.py" --model resnet50 --steps 3 --warmup 3 --no-latency > $O/prof$v.log 2>&1 || { tail -30 $O/prof$v.log; exit 1; }
python3 "$R/tools/rocprof_window.py" /tmp/prof_st$v --marker sgd --steps 2 --top 60 --seq > $O/window$v.md
echo "== stem=$v"; head -1 $O/window$v.md
awk -F'|' 'NF>4 && $5+0 > 40 {print}' $O/window$v.md | cut -c1-150 | head -20
done
