#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5l4
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_llm_gpu.py -k "swiglu or rmsnorm or linear or llama" > $O/pytest.log 2>&1 || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
PYTHONPATH=. timeout -k 10 120 python tools/probes/swiglu_t_bench.py 2>&1 | grep -v amdgpu.ids
for v in 1 0 1 0; do
PTO_SWIGLU_T=$v timeout -k 10 600 python bench.py --model llama3-8b --steps 10 --warmup 2 --no-latency > $O/llama_t$v.json 2> $O/llama_t$v.err || { tail -20 $O/llama_t$v.err; exit 1; }
python -c "import json; d=json.load(open('$O/llama_t$v.json')); print('swiglu_t=$v', d['value'], d['ms_per_step'])"
done
