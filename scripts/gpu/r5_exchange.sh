#!/bin/bash
# Round 5: the overlapped multi-GPU step with its whole exchange inside the
# next F12 launch.  DDP / graph / xGMI GPU tests, the world-1 step times of
# every schedule, and rocprofv3 kernel stats of the xGMI schedule.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
O=gpurun_out/r5x
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_xgmi_gpu.py tests/test_graph_gpu.py tests/test_ddp_gpu.py -v --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest.log | tail -2; grep FAILED $O/pytest.log | head
case $rc in 0|1) ;; *) echo "pytest rc=$rc"; exit $rc;; esac
timeout -k 10 300 python tools/ddp_step_bench.py --steps 2000 --warmup 200 > $O/ddp_step.json 2> $O/ddp_step.err || { tail -20 $O/ddp_step.err; exit 1; }
cat $O/ddp_step.json
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kst_x -o run -- python3 "$R/tools/ddp_step_bench.py" --steps 400 --warmup 50 --only xgmi > "$R/$O/prof.log" 2>&1 || { echo "rocprof rc=$?"; exit 1; }
f=$(find /tmp/kst_x -name "*kernel_stats.csv" | head -1)
python3 "$R/tools/kstats_table.py" "$f" | tee "$R/$O/kstats_xgmi.txt"
exit $rc
