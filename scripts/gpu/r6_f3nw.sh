#!/bin/bash
# Split fc1 forward: 4 / 8 / 16 waves per workgroup (PTO_FC1_NW), the
# kernel test under each, then interleaved 2000-step benches.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6_f3nw
mkdir -p $O
for v in 8 4 16; do
  PTO_FC1_NW=$v timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "fc1" -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -20 $O/pytest_$v.log; exit 1; }
  echo "nw=$v $(tail -1 $O/pytest_$v.log)"
done
for r in 1 2 3; do
  for v in 8 4 16; do
    PTO_FC1_NW=$v timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-latency > $O/b2000_${v}_$r.json 2>/dev/null || exit 1
    python -c "import json; a=json.load(open('$O/b2000_${v}_$r.json')); print('nw=$v', a['value'], a['ms_per_step'])"
  done
done
