#!/bin/bash
# Graphs warm-replayed once (default) vs twice at capture: the driver's
# 20-step command, interleaved, fresh process each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6_warm
mkdir -p $O
for r in 1 2 3 4; do
  for v in 1 2; do
    PTO_GRAPH_WARM=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-latency > $O/b20_${v}_$r.json 2>/dev/null || exit 1
    python -c "import json; b=json.load(open('$O/b20_${v}_$r.json')); print('warm=$v', b['value'], b['ms_per_step'])"
  done
done
