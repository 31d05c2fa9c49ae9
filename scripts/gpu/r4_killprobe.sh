#!/bin/bash
# the killed-peer CLI test with and without the overlapped xGMI schedule
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for ov in 1 0 1; do
  PTO_XGMI_OVERLAP=$ov timeout -k 10 200 python -u -m pytest tests/test_xgmi_gpu.py -k peer_killed -x -v --timeout 150 --timeout-method thread > gpurun_out/kill_ov$ov.log 2>&1
  echo "overlap=$ov rc=$?"; grep -E "passed|failed" gpurun_out/kill_ov$ov.log | tail -1
done
grep -B2 -A40 "rank 1:" gpurun_out/kill_ov1.log | head -80
