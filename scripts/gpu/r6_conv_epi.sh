#!/bin/bash
# Conv epilogue with 4-byte paired tile writes: 1x1 / 3x3 per-shape timing
# against the baseline library (PTO_HIP_LIB), numerics tests, ResNet-50 step
# with the owned 1x1 forward on / off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6_conv_epi
mkdir -p $O
BASE=$GRAFT_REPO_ROOT/pytorch_operator_1_amd/_lib/ab/libpto_hip_base.so
timeout -k 10 400 python -u -m pytest tests/test_conv1x1_fwd_gpu.py tests/test_conv3x3_gpu.py -v --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for lib in base new; do
  if [ $lib = base ]; then export PTO_HIP_LIB=$BASE; else unset PTO_HIP_LIB; fi
  timeout -k 10 300 python tools/conv1x1_bench.py > $O/c1_$lib.jsonl 2> $O/c1.err || { tail -20 $O/c1.err; exit 1; }
  timeout -k 10 300 python tools/conv3x3_bench.py --no-dgrad --variants 64:1 > $O/c3_$lib.jsonl 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
done
unset PTO_HIP_LIB
python - <<'PY'
import json
O='gpurun_out/r6_conv_epi'
b=[json.loads(l) for l in open(f'{O}/c1_base.jsonl')]; n=[json.loads(l) for l in open(f'{O}/c1_new.jsonl')]
for x,y in zip(b,n): print('1x1', x['shape'], 'miopen', y['miopen_fwd'], 'owned base', x['owned_fwd_stats'], 'new', y['owned_fwd_stats'])
for f in ('base','new'):
    print('3x3', f, [l.strip()[:160] for l in open(f'{O}/c3_{f}.jsonl')][-1])
PY
for v in 1 0; do
  PTO_CONV1X1_FWD=$v timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 --no-latency > $O/resnet_$v.json 2> $O/resnet_err || { tail -20 $O/resnet_err; exit 1; }
  python -c "import json; d=json.load(open('$O/resnet_$v.json')); print('conv1x1_fwd=$v', d['value'], d['ms_per_step'])"
done
