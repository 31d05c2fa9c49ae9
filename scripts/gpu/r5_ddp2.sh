#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_xgmi_gpu.py -k "bucketer" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 400 python bench.py --model resnet50 --steps 20 --warmup 5 --no-latency --force-ddp > $O/resnet_ddp.json 2> $O/resnet_ddp.err || { tail -20 $O/resnet_ddp.err; exit 1; }
cut -c1-200 $O/resnet_ddp.json
timeout -k 10 400 python bench.py --model resnet50 --steps 20 --warmup 5 --no-latency > $O/resnet.json 2> $O/resnet.err || { tail -20 $O/resnet.err; exit 1; }
cut -c1-200 $O/resnet.json
