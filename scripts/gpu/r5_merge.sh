#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5r
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_bn_gpu.py "tests/test_llm_gpu.py::test_resnet_trainer_steps" "tests/test_llm_gpu.py::test_resnet_graph_step_matches_eager" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
PYTHONPATH=. timeout -k 10 300 python tools/probes/graph_alias_probe.py 256 224 > $O/alias.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/alias.txt | tail -3
[ $rc -eq 0 ] || exit 1
for i in 1 2; do
  timeout -k 10 400 python bench.py --model resnet50 --steps 20 --warmup 5 --no-latency > $O/bench_m$i.json 2> $O/bench_m$i.err || { tail -20 $O/bench_m$i.err; exit 1; }
  cut -c1-200 $O/bench_m$i.json
done
timeout -k 10 400 python bench.py --model resnet50 --steps 20 --warmup 5 --no-latency --force-ddp > $O/bench_ddp.json 2> $O/bench_ddp.err || { tail -20 $O/bench_ddp.err; exit 1; }
cut -c1-200 $O/bench_ddp.json
