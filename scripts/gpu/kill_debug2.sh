#!/bin/bash
# Full GPU suite as the round check runs it, with replica stack dumps if the config-2 kill test stalls.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
PTO_PORT_RELEASE=${PTO_PORT_RELEASE:-1} PTO_TEST_KILL_TIMEOUT=100 PTO_TEST_DUMP_AFTER=${PTO_TEST_DUMP_AFTER:-45} timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/kill_debug2.log 2>&1
echo "rc=$?"
grep -E "passed|failed" gpurun_out/kill_debug2.log | tail -2
