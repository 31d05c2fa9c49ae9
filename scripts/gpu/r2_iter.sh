#!/bin/bash
# Iteration check: graph/kernel GPU tests, bench at 20 and 2000 steps, and a
# 2-rank DDP rehearsal on the one GPU (gloo rendezvous, same-device xGMI).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_graph_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/it_tests.log 2>&1 || { tail -40 gpurun_out/it_tests.log; exit 1; }
tail -3 gpurun_out/it_tests.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-latency > gpurun_out/it_b20.log 2>&1
grep -o '"value": [0-9.]*, "unit": "samples/s", "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*' gpurun_out/it_b20.log
timeout -k 10 200 python bench.py --no-latency > gpurun_out/it_b2000.log 2>&1
grep -o '"value": [0-9.]*, "unit": "samples/s", "n_gpus": 1, "steps": 2000, "warmup": 200, "ms_per_step": [0-9.]*' gpurun_out/it_b2000.log
if [ "${DDP:-1}" = "1" ]; then
PTO_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/it_ddp2.log 2>&1 || { tail -30 gpurun_out/it_ddp2.log; exit 1; }
grep -o '"value": [0-9.]*.*"grad_allreduce": {[^}]*}' gpurun_out/it_ddp2.log | cut -c1-600
fi
