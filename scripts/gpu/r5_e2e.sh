#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_e2e_gpu.py -s -v --timeout 420 --timeout-method thread > $O/e2e_all.log 2>&1
echo "rc=$?"
grep -E "PASSED|FAILED" $O/e2e_all.log
