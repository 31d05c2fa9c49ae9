#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for h in 1 0 0; do
  PTO_SYNTH_HOST=$h timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py -x -q -k deterministic --timeout 120 --timeout-method thread > gpurun_out/det_$h.log 2>&1 && echo "host=$h ok" || { echo "host=$h FAIL"; grep -E "^E .*diverged|^E .*differ|AssertionError" gpurun_out/det_$h.log | head -3; }
done
