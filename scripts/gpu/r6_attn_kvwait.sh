#!/bin/bash
# dK/dV producer loop: explicit K/V-fragment wait (PTO_ATTN_PC_KVWAIT=1,
# default) vs the old loop whose MFMAs waited on the next slice's loads.
# Interleaved A/B of the attention kernels, the attention GPU tests, then
# the Llama-3-8B step both ways.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6_attn_kvwait
mkdir -p $O
for r in 1 2; do
  for v in 0 1; do
    PTO_ATTN_PC_KVWAIT=$v timeout -k 10 120 python tools/attn_ab.py >> $O/attn_ab.jsonl 2>> $O/attn_ab.err || exit 1
  done
done
cat $O/attn_ab.jsonl
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py -v --timeout 150 --timeout-method thread > $O/pytest_attn.log 2>&1 || { tail -30 $O/pytest_attn.log; exit 1; }
tail -1 $O/pytest_attn.log
for v in 1 0; do
  PTO_ATTN_PC_KVWAIT=$v timeout -k 10 400 python bench.py --model llama3-8b --steps 10 --warmup 2 > $O/llama_kvw$v.json 2> $O/llama_kvw$v.err || { tail -20 $O/llama_kvw$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/llama_kvw$v.json')); print('kvwait=$v', d['value'], d['ms_per_step'])"
done
