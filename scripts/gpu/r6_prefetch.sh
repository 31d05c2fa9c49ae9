#!/bin/bash
# Next-batch prefetch in F4dx's extra workgroups (PTO_PREFETCH=1, default)
# vs none, interleaved: 2000-step bench and the driver's 20-step command;
# then the MNIST GPU tests that run F4dx (kernels, graphs, parity, DDP).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6_prefetch
mkdir -p $O
for r in 1 2; do
  for v in 1 0; do
    PTO_PREFETCH=$v timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-latency > $O/b2000_${v}_$r.json 2>/dev/null || exit 1
    PTO_PREFETCH=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/b20_${v}_$r.json 2>/dev/null || exit 1
    python -c "import json; a=json.load(open('$O/b2000_${v}_$r.json')); b=json.load(open('$O/b20_${v}_$r.json')); print('prefetch=$v', a['value'], a['ms_per_step'], '| driver cmd', b['value'], b['ms_per_step'])"
  done
done
timeout -k 10 700 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py tests/test_parity_long_gpu.py tests/test_ddp_gpu.py -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
