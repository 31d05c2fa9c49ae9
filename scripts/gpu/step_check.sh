#!/bin/bash
# MNIST step check: kernel / graph / DDP / xGMI GPU tests, the default bench,
# the DDP-schedule step time at world size 1, and rocprofv3 kernel stats of
# the one-process step (summary -> gpurun_out/step_kstats.txt).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py tests/test_ddp_gpu.py tests/test_xgmi_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_step.log 2>&1 || { tail -60 gpurun_out/pytest_step.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_step.log | tail -2
timeout -k 10 200 python bench.py --no-latency > gpurun_out/bench_step.json 2> gpurun_out/bench_step.err || { tail -20 gpurun_out/bench_step.err; exit 1; }
cut -c1-200 gpurun_out/bench_step.json
timeout -k 10 200 python tools/ddp_step_bench.py --steps 2000 --warmup 200 > gpurun_out/ddp_step.json 2> gpurun_out/ddp_step.err || { tail -20 gpurun_out/ddp_step.err; exit 1; }
cat gpurun_out/ddp_step.json
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kst_step -o run -- python3 "$R/bench.py" --steps 200 --warmup 20 --no-latency > "$R/gpurun_out/step_prof.log" 2>&1
f=$(find /tmp/kst_step -name "*kernel_stats.csv" | head -1)
python3 "$R/tools/kstats_table.py" "$f" | tee "$R/gpurun_out/step_kstats.txt"
