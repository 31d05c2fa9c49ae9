#!/bin/bash
# round-end check of the committed tree: every GPU test, smoke(), the default
# bench and the driver's 20-step command
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed|FAILED" gpurun_out/final/pytest_gpu.log | tail -8
case $rc in 0|1) ;; *) echo "pytest rc=$rc"; exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/final/bench_default.json 2> gpurun_out/final/bench_default.err || { tail -20 gpurun_out/final/bench_default.err; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/final/bench_driver.json 2> gpurun_out/final/bench_driver.err || { tail -20 gpurun_out/final/bench_driver.err; exit 1; }
for f in bench_default bench_driver; do python -c "import json; d=json.load(open('gpurun_out/final/$f.json')); print('$f', d['value'], d['ms_per_step'], d.get('submit_to_first_step_s'))"; done
exit $rc
