#!/bin/bash
# submit -> first step after dropping amdsmi (device_count) and GPU-generator
# seeding from the training image's start; then the default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/st
timeout -k 10 300 python tools/first_step_latency.py --gpu --runs 5 --zygote 1 > gpurun_out/st/latency5.jsonl 2> gpurun_out/st/latency5.err || { tail -20 gpurun_out/st/latency5.err; exit 1; }
cat gpurun_out/st/latency5.jsonl
timeout -k 10 300 python bench.py > gpurun_out/st/bench_default5.json 2> gpurun_out/st/bench_default5.err || { tail -20 gpurun_out/st/bench_default5.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/st/bench_default5.json')); print(d['value'], d['ms_per_step'], d.get('submit_to_first_step_s'), d['config']['final_loss'])"
