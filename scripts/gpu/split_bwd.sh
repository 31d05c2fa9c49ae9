#!/bin/bash
# Two-stream backward of the fused MNIST step: numerics, then bench on/off.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_split.log 2>&1 || { tail -60 gpurun_out/pytest_split.log; exit 1; }
tail -1 gpurun_out/pytest_split.log
for f in 1 0 1; do
  PTO_SPLIT_BWD=$f timeout -k 10 120 python bench.py --steps 3072 --warmup 320 > gpurun_out/split_$f.json 2>/dev/null
  echo "split_bwd=$f $(python -c "import json;d=json.load(open('gpurun_out/split_$f.json'));print(d['ms_per_step']*1e3,'us/step',d['value'])")"
done
