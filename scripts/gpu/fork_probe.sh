#!/bin/bash
# Cost of a side-stream fork/join inside the replayed MNIST graph.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for f in 0 1; do
  PTO_SPLIT_BWD=0 PTO_PROBE_FORK=$f timeout -k 10 120 python bench.py --steps 3072 --warmup 320 > gpurun_out/fork_$f.json 2>/dev/null
  echo "fork=$f $(python -c "import json;d=json.load(open('gpurun_out/fork_$f.json'));print(d['ms_per_step']*1e3,'us/step')")"
done
for u in 1; do
  PTO_SPLIT_BWD=0 PTO_PROBE_FORK=1 PTO_GRAPH_UNROLL=$u timeout -k 10 120 python bench.py --steps 1024 --warmup 64 > gpurun_out/fork_u$u.json 2>/dev/null
  echo "fork=1 unroll=$u $(python -c "import json;d=json.load(open('gpurun_out/fork_u$u.json'));print(d['ms_per_step']*1e3,'us/step')")"
done
