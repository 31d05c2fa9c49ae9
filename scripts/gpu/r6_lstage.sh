#!/bin/bash
# This step's labels staged by F12's last workgroup so F4dx's label load does
# not wait on a cursor load (PTO_LSTAGE=1, default) vs F4dx reading
# target[cursor] (0), interleaved; then every MNIST GPU test on the staged path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6_lstage
mkdir -p $O
for r in 1 2 3; do
  for v in 1 0; do
    PTO_LSTAGE=$v timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-latency > $O/b2000_${v}_$r.json 2>/dev/null || exit 1
    python -c "import json; a=json.load(open('$O/b2000_${v}_$r.json')); print('lstage=$v', a['value'], a['ms_per_step'])"
  done
done
PTO_LSTAGE=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/b20.json 2>/dev/null || exit 1
python -c "import json; b=json.load(open('$O/b20.json')); print('driver cmd', b['value'], b['ms_per_step'])"
PTO_LSTAGE=1 timeout -k 10 200 python tools/ddp_step_bench.py --steps 2000 > $O/ddp_step.json 2> $O/ddp_step.err || { tail -5 $O/ddp_step.err; exit 1; }
tail -c 400 $O/ddp_step.json; echo
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py tests/test_parity_long_gpu.py tests/test_ddp_gpu.py tests/test_xgmi_gpu.py -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
