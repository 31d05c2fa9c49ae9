#!/bin/bash
# CPU-only seeding in the fused trainer and the training image (no GPU generator touch):
# startup phases, submit -> first step, every GPU test, the default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/st
timeout -k 10 300 python tools/startup_probe.py > gpurun_out/st/startup4.json 2> gpurun_out/st/startup4.err || { tail -20 gpurun_out/st/startup4.err; exit 1; }
cat gpurun_out/st/startup4.json
timeout -k 10 200 python tools/ctor_probe.py > gpurun_out/st/ctor4.json 2> gpurun_out/st/ctor4.err || { tail -20 gpurun_out/st/ctor4.err; exit 1; }
cat gpurun_out/st/ctor4.json
timeout -k 10 300 python tools/first_step_latency.py --gpu --runs 3 --zygote 1 > gpurun_out/st/latency4.jsonl 2> gpurun_out/st/latency4.err || { tail -20 gpurun_out/st/latency4.err; exit 1; }
cat gpurun_out/st/latency4.jsonl
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/st/pytest_gpu4.log 2>&1
rc=$?
grep -E "passed|failed|FAILED" gpurun_out/st/pytest_gpu4.log | tail -8
case $rc in 0|1) ;; *) echo "pytest rc=$rc"; exit $rc;; esac
timeout -k 10 300 python bench.py > gpurun_out/st/bench_default4.json 2> gpurun_out/st/bench_default4.err || { tail -20 gpurun_out/st/bench_default4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/st/bench_default4.json')); print(d['value'], d['ms_per_step'], d.get('submit_to_first_step_s'), d['config']['final_loss'])"
exit $rc
