#!/bin/bash
# Round validation: smoke, every gpu test, default bench, rocprof of the bench.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -40 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -80 gpurun_out/pytest_gpu.log; exit 1; }
grep -E "passed|failed|submit ->" gpurun_out/pytest_gpu.log | tail -5
timeout -k 10 200 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
R="$GRAFT_REPO_ROOT"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_fused" -o run -- python3 "$R/bench.py" --steps 200 --warmup 20 --no-latency > "$R/gpurun_out/fused_prof.log" 2>&1
python3 "$R/tools/rocprof_summary.py" "$R/gpurun_out/prof_fused" --top 12
echo done
