#!/bin/bash
# A/B: dW1 tiles in their own blocks (0) vs done by the dgrad blocks (1):
# kernel tests, bench (2000 steps) and rocprof stats for each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in 1 0 1 0; do
  PTO_BWD_D_IN_B=$v timeout -k 10 200 python bench.py --no-latency > gpurun_out/dinb_$v.json 2> gpurun_out/dinb_$v.err || { tail -5 gpurun_out/dinb_$v.err; exit 1; }
  echo "d_in_b=$v $(cut -c1-140 gpurun_out/dinb_$v.json)"
done
PTO_BWD_D_IN_B=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dinb.log 2>&1; echo "tests(d_in_b=1) rc=$?"; tail -2 gpurun_out/pytest_dinb.log
cd /tmp
for v in 0 1; do
  rm -rf /tmp/kst_d$v
  PTO_BWD_D_IN_B=$v timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kst_d$v -o run -- python3 "$R/bench.py" --steps 200 --warmup 20 --no-latency > "$R/gpurun_out/dinb_prof_$v.log" 2>&1 || exit 1
  f=$(find /tmp/kst_d$v -name "*kernel_stats.csv" | head -1)
  echo "== d_in_b=$v"; python3 "$R/tools/kstats_table.py" "$f" --top 5
done
