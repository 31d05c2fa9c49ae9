#!/bin/bash
# fc1 folded into F12: GPU tests, the N=1 bench with and without it, the
# world-1 DDP step, and rocprofv3 kernel stats of the fused step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
O=gpurun_out/r5f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py tests/test_parity_long_gpu.py tests/test_ddp_gpu.py -v -s --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest.log | tail -2; grep FAILED $O/pytest.log | head
case $rc in 0) ;; *) echo "pytest rc=$rc"; exit 1;; esac
for v in 1 0 1 0; do
PTO_FUSE_FC1=$v timeout -k 10 300 python bench.py --no-latency > $O/bench_f$v.json 2> $O/bench_f$v.err || { tail -20 $O/bench_f$v.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_f$v.json')); print('fuse_fc1=$v', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-latency > $O/bench_drv.json 2> $O/bench_drv.err || { tail -20 $O/bench_drv.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_drv.json')); print('driver-cmd', d['value'], d['ms_per_step'])"
timeout -k 10 300 python tools/ddp_step_bench.py --steps 2000 --warmup 200 > $O/ddp_step.json 2> $O/ddp_step.err || { tail -20 $O/ddp_step.err; exit 1; }
grep '^{' $O/ddp_step.json
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kst_f -o run -- python3 "$R/bench.py" --steps 400 --warmup 50 --no-latency > "$R/$O/prof.log" 2>&1 || { echo "rocprof rc=$?"; exit 1; }
f=$(find /tmp/kst_f -name "*kernel_stats.csv" | head -1)
python3 "$R/tools/kstats_table.py" "$f" > "$R/$O/kstats.txt"
head -12 "$R/$O/kstats.txt"
