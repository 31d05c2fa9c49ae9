#!/bin/bash
# 1x1 forward: single LDS buffer (more workgroups per CU) vs double buffer,
# per shape against CK; numerics tests; ResNet-50 with the owned 1x1
# forward on / off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6_conv1x1_nb
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_conv1x1_fwd_gpu.py -v --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python tools/conv1x1_bench.py > $O/bench.jsonl 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json
for l in open('$O/bench.jsonl'):
    d=json.loads(l); print(d['shape'], 'miopen', d['miopen_fwd'], 'nb2+stats', d['owned_fwd_stats_nb2'], 'persist+stats', d['owned_fwd_stats_nb3'], 'nb1', d['owned_fwd'], 'nb1+stats', d['owned_fwd_stats'], 'err nb2/3/1', round(d['owned_err_nb2'],4), round(d['owned_err_nb3'],4), round(d['owned_err'],4))
"
for v in 1 0; do
  PTO_CONV1X1_FWD=$v timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 --no-latency > $O/resnet_$v.json 2> $O/resnet_err || { tail -20 $O/resnet_err; exit 1; }
  python -c "import json; d=json.load(open('$O/resnet_$v.json')); print('conv1x1_fwd=$v', d['value'], d['ms_per_step'])"
done
