#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
PTO_TEST_KILL_TIMEOUT=240 PTO_TEST_DUMP_AFTER=150 timeout -k 10 500 python -u -m pytest tests/test_e2e_gpu.py -x -v -k config2 --timeout 400 --timeout-method thread > gpurun_out/kill_debug.log 2>&1 || { tail -150 gpurun_out/kill_debug.log; exit 1; }
grep -E "passed|failed" gpurun_out/kill_debug.log | tail -2
