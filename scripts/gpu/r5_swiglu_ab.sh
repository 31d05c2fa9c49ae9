#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5a
mkdir -p $O
for v in 0 1 0 1; do
PTO_SWIGLU_T=$v timeout -k 10 600 python bench.py --model llama3-8b --steps 10 --warmup 2 --no-latency > $O/llama_t$v.json 2> $O/llama_t$v.err || { tail -20 $O/llama_t$v.err; exit 1; }
python -c "import json; d=json.load(open('$O/llama_t$v.json')); print('swiglu_t=$v', d['value'], d['ms_per_step'])"
done
