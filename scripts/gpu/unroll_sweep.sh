#!/bin/bash
# Steps per HIP-graph replay (PTO_GRAPH_UNROLL) vs MNIST step time.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for u in 1 8 32 64; do
  PTO_GRAPH_UNROLL=$u timeout -k 10 120 python bench.py --steps 3072 --warmup 320 > gpurun_out/unroll_$u.json 2>/dev/null
  echo "unroll=$u $(python -c "import json;d=json.load(open('gpurun_out/unroll_$u.json'));print(d['ms_per_step']*1e3,'us/step',d['value'])")"
done
