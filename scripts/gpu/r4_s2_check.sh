#!/bin/bash
# Session-2 re-entry check of HEAD: smoke, every gpu test, default bench
# (the driver's command), then the world-1 DDP schedule costs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -40 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed|FAILED" gpurun_out/pytest_gpu.log | tail -12
case $rc in 0|1) ;; *) echo "pytest rc=$rc"; exit $rc;; esac
for i in 1 2 3; do
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_drv$i.json 2> gpurun_out/bench_drv$i.err || { tail -20 gpurun_out/bench_drv$i.err; exit 1; }
cut -c1-200 gpurun_out/bench_drv$i.json
done
timeout -k 10 200 python tools/ddp_step_bench.py --steps 2000 --warmup 200 > gpurun_out/ddp_step.json 2> gpurun_out/ddp_step.err || { tail -20 gpurun_out/ddp_step.err; exit 1; }
cat gpurun_out/ddp_step.json
exit $rc
