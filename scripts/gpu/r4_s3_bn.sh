#!/bin/bash
# fused BN kernels on ResNet-50 shapes: bn_bench + per-kernel rocprof stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/bn
timeout -k 10 300 python -u -m pytest tests/test_bn_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/bn/pytest.log 2>&1 || { tail -30 gpurun_out/bn/pytest.log; exit 1; }
tail -1 gpurun_out/bn/pytest.log
timeout -k 10 300 python tools/bn_bench.py > gpurun_out/bn/bench.txt 2> gpurun_out/bn/bench.err || { tail -20 gpurun_out/bn/bench.err; exit 1; }
cat gpurun_out/bn/bench.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/bn/prof" -o bn -- python3 "$GRAFT_REPO_ROOT/tools/bn_bench.py" > "$GRAFT_REPO_ROOT/gpurun_out/bn/prof.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/bn/prof.log"; exit 1; }
find "$GRAFT_REPO_ROOT/gpurun_out/bn/prof" -name "*kernel_stats.csv" | head -3
cd "$GRAFT_REPO_ROOT"
( while sleep 20; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u bench.py --model resnet50 --steps 20 --warmup 3 > gpurun_out/bn/resnet.json 2> gpurun_out/bn/resnet.err || { tail -20 gpurun_out/bn/resnet.err; exit 1; }
cat gpurun_out/bn/resnet.json
