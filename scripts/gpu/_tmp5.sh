set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_xgmi_gpu.py tests/test_ddp_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_xgmi.log 2>&1 || { tail -60 gpurun_out/pytest_xgmi.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_xgmi.log | tail -2
timeout -k 10 200 python tools/ddp_step_bench.py --steps 2000 --warmup 200 > gpurun_out/ddp_step.json 2> gpurun_out/ddp_step.err || { tail -20 gpurun_out/ddp_step.err; exit 1; }
cat gpurun_out/ddp_step.json
