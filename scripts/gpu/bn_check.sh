#!/bin/bash
# Fused BN: numerics tests, then the ResNet-50 bench (fused vs MIOpen BN).
# SKIP_TESTS=1: benches only.  MIOpen find runs silently for minutes during
# the warmup, hence the heartbeat.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
( while sleep 30; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 300 python -u -m pytest tests/test_bn_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_bn.log 2>&1 || { tail -60 gpurun_out/pytest_bn.log; exit 1; }
  grep -E "passed|failed" gpurun_out/pytest_bn.log | tail -1
fi
for f in ${BN_MODES:-1 0}; do
  PTO_FUSED_BN=$f timeout -k 10 400 python -u bench.py --model resnet50 --steps 20 --warmup 5 --breakdown > gpurun_out/resnet_bn$f.json 2> gpurun_out/resnet_bn$f.err || { tail -20 gpurun_out/resnet_bn$f.err; exit 1; }
  echo "fused_bn=$f $(cut -c1-170 gpurun_out/resnet_bn$f.json) $(grep 'phase ms' gpurun_out/resnet_bn$f.err)"
done
