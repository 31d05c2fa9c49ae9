#!/bin/bash
# Round 6 check of the committed tree: every GPU test, smoke(), the default
# bench and the driver's 20-step command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/check6
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest_gpu.log | tail -2; grep FAILED $O/pytest_gpu.log | head
case $rc in 0|1) ;; *) echo "pytest rc=$rc"; exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
for f in bench_default bench_driver; do python -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'], d.get('submit_to_first_step_s'))"; done
exit $rc
