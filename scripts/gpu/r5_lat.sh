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
