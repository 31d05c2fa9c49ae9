#!/bin/bash
# Reproduce the config-2 kill/rejoin hang with the test files that run before it, stacks dumped after 60 s.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
PTO_TEST_KILL_TIMEOUT=120 PTO_TEST_DUMP_AFTER=60 timeout -k 10 600 python -u -m pytest tests/test_attention_gpu.py tests/test_bn_gpu.py tests/test_ddp_gpu.py tests/test_e2e_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/kill_debug.log 2>&1
echo "rc=$?"
grep -E "passed|failed" gpurun_out/kill_debug.log | tail -2
