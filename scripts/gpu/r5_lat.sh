#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5l
mkdir -p $O
for n in 1 2; do
timeout -k 10 200 python -c "
import bench, json
r = bench.measure_submit_to_first_step(gpu=True, replicas=$n, timeout=150)
print(json.dumps(r))
" > $O/lat$n.json 2> $O/lat$n.err || { tail -5 $O/lat$n.err; exit 1; }
cat $O/lat$n.json
done
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_e2e_gpu.py > $O/e2e.log 2>&1 || { tail -30 $O/e2e.log; exit 1; }
tail -3 $O/e2e.log
