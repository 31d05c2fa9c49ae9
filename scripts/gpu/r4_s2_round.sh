#!/bin/bash
# Full round check of HEAD: smoke, every GPU test, the driver's bench
# command x3, 2000-step bench, rocprofv3 kernel stats of the N=1 step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rc/smoke.log 2>&1 || { tail -40 gpurun_out/rc/smoke.log; exit 1; }
tail -1 gpurun_out/rc/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/rc/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed|FAILED" gpurun_out/rc/pytest_gpu.log | tail -8
case $rc in 0|1) ;; *) echo "pytest rc=$rc"; exit $rc;; esac
for i in 1 2 3; do
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/rc/bench_drv$i.json 2> gpurun_out/rc/bench_drv$i.err || { tail -20 gpurun_out/rc/bench_drv$i.err; exit 1; }
cut -c1-160 gpurun_out/rc/bench_drv$i.json
done
timeout -k 10 200 python bench.py --no-latency > gpurun_out/rc/bench_2000.json 2> gpurun_out/rc/bench_2000.err || { tail -20 gpurun_out/rc/bench_2000.err; exit 1; }
cut -c1-160 gpurun_out/rc/bench_2000.json
cd /tmp && rm -rf /tmp/kst1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kst1 -o run -- python3 "$R/bench.py" --steps 400 --warmup 40 --no-latency > "$R/gpurun_out/rc/prof.log" 2>&1 || exit 1
f=$(find /tmp/kst1 -name "*kernel_stats.csv" | head -1)
python3 "$R/tools/kstats_table.py" "$f" | tee "$R/gpurun_out/rc/kstats_n1.txt"
exit $rc
