#!/bin/bash
# conv1 gradient replicas (k_bwd_all's B-role atomics spread over nrep
# copies; F12's lazy update and F4dx's commit read all of them): 8 / 4 / 16,
# interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6_c1rep
mkdir -p $O
for r in 1 2; do
  for v in 8 4 16 2; do
    PTO_C1_REPLICAS=$v timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-latency > $O/b2000_${v}_$r.json 2>/dev/null || exit 1
    python -c "import json; a=json.load(open('$O/b2000_${v}_$r.json')); print('nrep=$v', a['value'], a['ms_per_step'])"
  done
done
