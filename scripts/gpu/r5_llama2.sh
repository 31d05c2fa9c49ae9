#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5l3
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_llm_gpu.py tests/test_linear_tw.py > $O/pytest.log 2>&1 || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log


for i in 1 2; do
timeout -k 10 600 python bench.py --model llama3-8b --steps 10 --warmup 2 --no-latency > $O/llama$i.json 2> $O/llama$i.err || { tail -20 $O/llama$i.err; exit 1; }
python -c "import json; d=json.load(open('$O/llama$i.json')); print('llama', d['value'], d['ms_per_step'], d['config'].get('mfu'))"
done
