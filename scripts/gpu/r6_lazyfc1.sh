#!/bin/bash
# fc1.weight's update (dW1 tiles + SGD) as extra workgroups of the next
# step's F12 (PTO_LAZY_FC1=1, default) vs k_bwd_all's D role (0),
# interleaved; then every MNIST GPU test on the lazy path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6_lazyfc1
mkdir -p $O
for r in 1 2 3; do
  for v in 1 0; do
    PTO_LAZY_FC1=$v timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-latency > $O/b2000_${v}_$r.json 2>/dev/null || exit 1
    python -c "import json; a=json.load(open('$O/b2000_${v}_$r.json')); print('lazyfc1=$v', a['value'], a['ms_per_step'])"
  done
done
for v in 1 0; do
PTO_LAZY_FC1=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-latency > $O/b20_$v.json 2>/dev/null || exit 1
python -c "import json; b=json.load(open('$O/b20_$v.json')); print('driver cmd lazyfc1=$v', b['value'], b['ms_per_step'])"
done
PTO_LAZY_FC1=1 timeout -k 10 200 python tools/ddp_step_bench.py --steps 2000 > $O/ddp_step.json 2> $O/ddp_step.err || { tail -5 $O/ddp_step.err; exit 1; }
tail -c 400 $O/ddp_step.json; echo
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py tests/test_parity_long_gpu.py tests/test_ddp_gpu.py tests/test_xgmi_gpu.py -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
