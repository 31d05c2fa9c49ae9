#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5r
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_bn_gpu.py "tests/test_llm_gpu.py::test_resnet_trainer_steps" "tests/test_llm_gpu.py::test_resnet_graph_step_matches_eager" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for g in 0 1; do
  PTO_STEP_GRAPH=$g timeout -k 10 400 python bench.py --model resnet50 --steps 20 --warmup 5 --no-latency > $O/bench_g$g.json 2> $O/bench_g$g.err || { tail -20 $O/bench_g$g.err; exit 1; }
  cut -c1-250 $O/bench_g$g.json
done
