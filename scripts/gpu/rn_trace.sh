#!/bin/bash
# Kernel trace of a short ResNet-50 bench run, BN kernels grouped by grid size.
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rn
( while sleep 20; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export TMPDIR=/tmp
cd /tmp
rm -rf /tmp/rnt
timeout -s KILL 900 rocprofv3 --kernel-trace --output-format csv -d /tmp/rnt -o run -- python3 "$R/bench.py" --model resnet50 --steps 3 --warmup 3 > "$R/gpurun_out/rn/trace.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/rn/trace.log"; exit 1; }
f=$(find /tmp/rnt -name "*kernel_trace.csv" | head -1)
python3 "$R/tools/trace_by_grid.py" "$f" --filter k_bn --top 60 > "$R/gpurun_out/rn/bn_by_grid.txt"
python3 "$R/tools/trace_by_grid.py" "$f" --top 30 > "$R/gpurun_out/rn/all_by_grid.txt"
head -5 "$R/gpurun_out/rn/all_by_grid.txt"
