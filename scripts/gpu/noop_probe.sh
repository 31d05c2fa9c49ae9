#!/bin/bash
# Cost of one launch boundary inside the replayed MNIST graph: k empty
# kernels after each of the 6 phase launches.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 0 1 2; do
  for b in 1 256; do
    PTO_PROBE_NOOPS=$k PTO_PROBE_BLOCKS=$b timeout -k 10 120 python bench.py --steps 3000 --warmup 300 > gpurun_out/noop_${k}_${b}.json 2>/dev/null
    echo "noops=$k blocks=$b $(python -c "import json;d=json.load(open('gpurun_out/noop_${k}_${b}.json'));print(d['ms_per_step']*1e3,'us/step')")"
    [ $k = 0 ] && break
  done
done
