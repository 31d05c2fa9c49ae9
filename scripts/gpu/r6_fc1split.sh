#!/bin/bash
# fc1 forward split-K over two workgroups per tile with F4dx forming
# relu(h + b1) from the atomically summed halves (PTO_FC1_SPLIT=1, default) vs one 16-wave workgroup per
# tile with the bias/ReLU epilogue (0), interleaved; F3 phase stamps both
# ways; then every MNIST GPU test on the split path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6_fc1split${TAG:-}
mkdir -p $O
for v in 1 0; do
PTO_FC1_SPLIT=$v timeout -k 10 300 python tools/bwd_phases_probe.py --fwd --reps 30 > $O/fwd_phases_$v.txt 2>&1 || { tail -20 $O/fwd_phases_$v.txt; exit 1; }
grep "^F3" $O/fwd_phases_$v.txt
done
for r in 1 2 3; do
  for v in 1 0; do
    PTO_FC1_SPLIT=$v timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-latency > $O/b2000_${v}_$r.json 2>/dev/null || exit 1
    python -c "import json; a=json.load(open('$O/b2000_${v}_$r.json')); print('fc1split=$v', a['value'], a['ms_per_step'])"
  done
done
for v in 1 0; do
PTO_FC1_SPLIT=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-latency > $O/b20_$v.json 2>/dev/null || exit 1
python -c "import json; b=json.load(open('$O/b20_$v.json')); print('driver cmd fc1split=$v', b['value'], b['ms_per_step'])"
done
PTO_FC1_SPLIT=1 timeout -k 10 200 python tools/ddp_step_bench.py --steps 2000 > $O/ddp_step.json 2> $O/ddp_step.err || { tail -5 $O/ddp_step.err; exit 1; }
tail -c 400 $O/ddp_step.json; echo
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py tests/test_parity_long_gpu.py tests/test_ddp_gpu.py tests/test_xgmi_gpu.py -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
