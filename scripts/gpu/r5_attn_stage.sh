#!/bin/bash
# Attention forward / dQ with the K/V staging split across the barrier
# (libpto_hip_new.so) vs the committed kernels (libpto_hip_base.so):
# numerics, then kernel and Llama-3-8B step A/B on one box.  Build the two
# libraries first (python -c 'import __graft_entry__ as g; g.build()' on
# each tree, copied to _lib/libpto_hip_{new,base}.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${R5AS_OUT:-r5as}
mkdir -p $O
L=pytorch_operator_1_amd/_lib
cp $L/libpto_hip_new.so $L/libpto_hip.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do for v in new base; do
cp $L/libpto_hip_$v.so $L/libpto_hip.so
ITERS=30 timeout -k 10 120 python tools/attn_ab.py 2>/dev/null | sed "s/^/$v /" | tee -a $O/ab.txt
done; done
for v in new base new base; do
cp $L/libpto_hip_$v.so $L/libpto_hip.so
timeout -k 10 600 python bench.py --model llama3-8b --steps 10 --warmup 2 --no-latency > $O/llama_$v.json 2> $O/llama_$v.err || { tail -20 $O/llama_$v.err; exit 1; }
python -c "import json; d=json.load(open('$O/llama_$v.json')); print('llama $v', d['value'], d['ms_per_step'])"
done
cp $L/libpto_hip_new.so $L/libpto_hip.so
