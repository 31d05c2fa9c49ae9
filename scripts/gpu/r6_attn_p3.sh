#!/bin/bash
# dK/dV: 12-wave two-producer kernel (PTO_ATTN_DKDV_PC=2) vs the 8-wave
# producer/consumer kernel (1), interleaved; attention GPU tests on the new
# kernel; Llama-3-8B step both ways.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6_attn_p3
mkdir -p $O
PTO_ATTN_DKDV_PC=2 timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py -v --timeout 150 --timeout-method thread > $O/pytest_attn_p3.log 2>&1 || { tail -30 $O/pytest_attn_p3.log; exit 1; }
tail -1 $O/pytest_attn_p3.log
for r in 1 2; do
  for v in 1 2; do
    PTO_ATTN_DKDV_PC=$v timeout -k 10 120 python tools/attn_ab.py >> $O/attn_ab.jsonl 2>> $O/attn_ab.err || exit 1
  done
done
cat $O/attn_ab.jsonl
for v in 2 1; do
  PTO_ATTN_DKDV_PC=$v timeout -k 10 400 python bench.py --model llama3-8b --steps 10 --warmup 2 > $O/llama_pc$v.json 2> $O/llama_pc$v.err || { tail -20 $O/llama_pc$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/llama_pc$v.json')); print('dkdv_pc=$v', d['value'], d['ms_per_step'])"
done
