#!/bin/bash
# Next batch staged by F4dx into a fixed buffer that F12 reads without the
# cursor (PTO_XSTAGE=1, default) vs F12 reading dataset[cursor] (0),
# interleaved; then every MNIST GPU test (kernels, graphs, parity, DDP, xGMI,
# e2e) on the staged path, and the 2-rank partitioned rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6_xstage
mkdir -p $O
for r in 1 2; do
  for v in 1 0; do
    PTO_XSTAGE=$v timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-latency > $O/b2000_${v}_$r.json 2>/dev/null || exit 1
    PTO_XSTAGE=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/b20_${v}_$r.json 2>/dev/null || exit 1
    python -c "import json; a=json.load(open('$O/b2000_${v}_$r.json')); b=json.load(open('$O/b20_${v}_$r.json')); print('xstage=$v', a['value'], a['ms_per_step'], '| driver cmd', b['value'], b['ms_per_step'])"
  done
done
PTO_XSTAGE=1 timeout -k 10 200 python tools/ddp_step_bench.py --steps 2000 > $O/ddp_step.json 2> $O/ddp_step.err || { tail -5 $O/ddp_step.err; exit 1; }
tail -c 400 $O/ddp_step.json; echo
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py tests/test_parity_long_gpu.py tests/test_ddp_gpu.py tests/test_xgmi_gpu.py -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
PTO_BACKEND=gloo PTO_CU_PARTITION=1 timeout -k 10 300 python bench.py --gpus 2 --steps 200 --warmup 5 --no-latency > $O/reh2.json 2> $O/reh2.err || { tail -20 $O/reh2.err; exit 1; }
python -c "import json; d=json.loads([l for l in open('$O/reh2.json') if l.startswith('{')][0]); print('reh2', d['value'], d['ms_per_step'], d.get('ranks_bit_identical'), d['config']['grad_allreduce'].get('overlap'))"
