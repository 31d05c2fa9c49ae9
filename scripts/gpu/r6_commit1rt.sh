#!/bin/bash
# conv1 commit (closing launch of every run, F4dx's commit workgroup, k_ddp_sgd)
# with all loads in one round trip vs a build of the previous tree
# (PTO_HIP_LIB), interleaved; then the MNIST GPU tests on the new library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6_commit1rt
mkdir -p $O
BASE=$GRAFT_REPO_ROOT/pytorch_operator_1_amd/_lib/ab/libpto_hip_base.so
for r in 1 2 3 4; do
  PTO_HIP_LIB=$BASE timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-latency > $O/b20_base_$r.json 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-latency > $O/b20_new_$r.json 2>/dev/null || exit 1
  python -c "import json; a=json.load(open('$O/b20_base_$r.json')); b=json.load(open('$O/b20_new_$r.json')); print('driver base', a['value'], '| new', b['value'])"
done
for r in 1 2; do
  PTO_HIP_LIB=$BASE timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-latency > $O/b2000_base_$r.json 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-latency > $O/b2000_new_$r.json 2>/dev/null || exit 1
  python -c "import json; a=json.load(open('$O/b2000_base_$r.json')); b=json.load(open('$O/b2000_new_$r.json')); print('2000 base', a['ms_per_step'], '| new', b['ms_per_step'])"
done
timeout -k 10 200 python tools/ddp_step_bench.py --steps 2000 > $O/ddp_step.json 2> $O/ddp_step.err || { tail -5 $O/ddp_step.err; exit 1; }
tail -c 400 $O/ddp_step.json; echo
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py tests/test_parity_long_gpu.py tests/test_ddp_gpu.py tests/test_xgmi_gpu.py -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
