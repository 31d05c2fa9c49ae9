#!/bin/bash
# MFMA stem conv: GPU tests (BN/pool/conv1x1/stem + ResNet trainer), the
# ResNet-50 bench with and without it, and a kernel window of the step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
O=gpurun_out/r5st
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_bn_gpu.py "tests/test_llm_gpu.py::test_resnet_trainer_steps" "tests/test_llm_gpu.py::test_resnet_graph_step_matches_eager" > $O/pytest.log 2>&1 || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in 1 0 1 0; do
PTO_STEM=$v timeout -k 10 400 python bench.py --model resnet50 --steps 20 --warmup 5 --no-latency > $O/bench_s$v.json 2> $O/bench_s$v.err || { tail -20 $O/bench_s$v.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_s$v.json')); print('stem=$v', d['value'], d['ms_per_step'])"
done
