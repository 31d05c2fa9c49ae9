#!/bin/bash
# Round validation: smoke, every gpu test (kernel numerics first, the
# multi-process operator tests last -- tests/conftest.py), default bench.
# Usage: round_check.sh [--no-x]
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
X="-x"; [ "$1" = "--no-x" ] && X=""
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -40 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
rc=0
timeout -k 10 1000 python -u -m pytest tests -m gpu $X -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || rc=$?
grep -E "passed|failed|FAILED|submit ->" gpurun_out/pytest_gpu.log | tail -12
case $rc in 0|1) ;; *) echo "pytest rc=$rc"; exit $rc;; esac
timeout -k 10 200 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
exit $rc
