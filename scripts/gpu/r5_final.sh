#!/bin/bash
# Round-5 check of the committed tree: every GPU test, smoke(), the default
# bench, the driver's 20-step command, and a 2-rank self-launched rehearsal
# (two ranks sharing the one GPU, gloo) with its N>1 JSON evidence, then
# the ResNet-50 and Llama-3-8B benches (BASELINE configs 3-4).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/final5
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -v -s --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest_gpu.log | tail -2; grep FAILED $O/pytest_gpu.log | head
case $rc in 0|1) ;; *) echo "pytest rc=$rc"; exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
for f in bench_default bench_driver; do python -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'], d.get('submit_to_first_step_s'))"; done
PTO_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 200 --warmup 5 > $O/reh2.json 2> $O/reh2.err || { tail -30 $O/reh2.err; exit 1; }
python -c "import json; d=json.loads([l for l in open('$O/reh2.json') if l.startswith('{')][0]); print('reh2', d['value'], d['ms_per_step'], d.get('submit_to_first_step_s'), d.get('ranks_bit_identical'), d['config']['grad_allreduce'].get('schedule_autotune', {}).get('kept'))"
for m in resnet50 llama3-8b; do
timeout -k 10 600 python bench.py --model $m --steps 20 --warmup 5 --no-latency > $O/bench_$m.json 2> $O/bench_$m.err || { tail -20 $O/bench_$m.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_$m.json')); print('$m', d['value'], d['ms_per_step'])"
done
exit $rc
