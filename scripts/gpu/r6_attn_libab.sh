#!/bin/bash
# Attention kernels: the current library vs a baseline build
# (pytorch_operator_1_amd/_lib/ab/libpto_hip_base.so, PTO_HIP_LIB),
# interleaved, at the Llama-3-8B shape; then the attention GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6_attn_libab
mkdir -p $O
BASE=$GRAFT_REPO_ROOT/pytorch_operator_1_amd/_lib/ab/libpto_hip_base.so
for r in 1 2 3; do
  PTO_HIP_LIB=$BASE timeout -k 10 120 python tools/attn_ab.py | sed 's/^/base /' >> $O/attn_ab.txt || exit 1
  timeout -k 10 120 python tools/attn_ab.py | sed 's/^/new  /' >> $O/attn_ab.txt || exit 1
done
cat $O/attn_ab.txt
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py -v --timeout 150 --timeout-method thread > $O/pytest_attn.log 2>&1 || { tail -30 $O/pytest_attn.log; exit 1; }
tail -1 $O/pytest_attn.log
