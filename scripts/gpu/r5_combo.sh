#!/bin/bash
# Early barrier-0 arrival + transposed SwiGLU backward: GPU tests, world-1
# DDP step with/without the early arrival, F12 phase probe, Llama-3-8B bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_llm_gpu.py tests/test_linear_tw.py tests/test_xgmi_gpu.py tests/test_graph_gpu.py tests/test_ddp_gpu.py -v -s --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest.log | tail -2; grep FAILED $O/pytest.log | head
case $rc in 0) ;; *) echo "pytest rc=$rc"; exit 1;; esac
for ea in 1 0; do
PTO_EARLY_ARRIVAL=$ea timeout -k 10 300 python tools/ddp_step_bench.py --steps 2000 --warmup 200 > $O/ddp_step_ea$ea.json 2> $O/ddp_step_ea$ea.err || { tail -20 $O/ddp_step_ea$ea.err; exit 1; }
echo "early_arrival=$ea $(grep '^{' $O/ddp_step_ea$ea.json)"
done
timeout -k 10 300 python tools/exchange_phases_probe.py > $O/phases.json 2> $O/phases.err || { tail -20 $O/phases.err; exit 1; }
grep '^{' $O/phases.json
timeout -k 10 600 python bench.py --model llama3-8b --steps 10 --warmup 2 --no-latency > $O/llama.json 2> $O/llama.err || { tail -20 $O/llama.err; exit 1; }
cut -c1-220 $O/llama.json
