#!/bin/bash
# Round 5: large-model configs -- ResNet-50 1x1-conv GEMM path A/B, the DDP
# path at world 1 (--force-ddp) for ResNet-50 and Llama-3-8B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5m
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_bn_gpu.py -v --timeout 300 --timeout-method thread > $O/pytest_bn.log 2>&1
echo "bn tests rc=$?"; grep -E "passed|failed" $O/pytest_bn.log | tail -1; grep FAILED $O/pytest_bn.log | head -5
for mode in 1 0; do
  PTO_CONV1X1_GEMM=$mode timeout -k 10 400 python bench.py --model resnet50 --steps 20 --warmup 5 > $O/resnet_gemm$mode.json 2> $O/resnet_gemm$mode.err || { echo "resnet gemm=$mode failed"; tail -5 $O/resnet_gemm$mode.err; }
  python -c "import json; d=json.load(open('$O/resnet_gemm$mode.json')); print('resnet gemm=$mode', d['value'], d['ms_per_step'])" || true
done
timeout -k 10 400 python bench.py --model resnet50 --steps 20 --warmup 5 --force-ddp > $O/resnet_ddp.json 2> $O/resnet_ddp.err || { tail -5 $O/resnet_ddp.err; }
python -c "import json; d=json.load(open('$O/resnet_ddp.json')); print('resnet force-ddp', d['value'], d['ms_per_step'], d['config']['grad_allreduce'].get('transport'), d['config'].get('bucket_mb'))" || true
timeout -k 10 600 python bench.py --model llama3-8b --steps 10 --warmup 2 --force-ddp > $O/llama_ddp.json 2> $O/llama_ddp.err || { tail -5 $O/llama_ddp.err; }
python -c "import json; d=json.load(open('$O/llama_ddp.json')); c=d['config']; print('llama force-ddp', d['value'], d['ms_per_step'], c['grad_allreduce'].get('transport'), c.get('bucket_mb'), c.get('peak_mem_gb'), c.get('projected_dp8_peak_gb'))" || true
