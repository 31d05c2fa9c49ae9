#!/bin/bash
# dK/dV kernel A/B: producer-consumer 8-wave kernel vs the 4-wave kernel; attention
# numerics under each.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 1 0 1 0; do
  PTO_ATTN_DKDV_PC=$v timeout -k 10 120 python tools/attn_ab.py | tee -a gpurun_out/attn_ab.jsonl
done
for v in 1 0; do
  PTO_ATTN_DKDV_PC=$v timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_pytest_$v.log 2>&1 || { tail -30 gpurun_out/attn_pytest_$v.log; exit 1; }
  tail -1 gpurun_out/attn_pytest_$v.log
done
