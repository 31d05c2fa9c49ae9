#!/bin/bash
# Round 6: ResNet-50 with the owned 3x3 conv (fwd + stride-1 dgrad + BN
# statistics epilogue): GPU tests touching the model, then the bench A/B
# (PTO_CONV3X3=1 vs 0), interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6resnet
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_conv3x3_gpu.py tests/test_bn_gpu.py tests/test_llm_gpu.py -k "conv3x3 or resnet or conv1x1 or bn_act or stem" -v -x --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest.log | tail -2; grep FAILED $O/pytest.log | head
[ $rc -eq 0 ] || { tail -40 $O/pytest.log; exit $rc; }
for v in 1 0 1 0; do
PTO_CONV3X3=$v timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 --no-latency > $O/bench_c3_$v.json 2> $O/bench_c3_$v.err || { tail -20 $O/bench_c3_$v.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c3_$v.json')); print('conv3x3=$v', d['value'], d['ms_per_step'])"
done
