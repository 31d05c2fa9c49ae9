#!/bin/bash
# Round 6: BASELINE configs 3-4 on the current tree -- Llama-3-8B and
# ResNet-50 (20 timed steps), and both with the DDP path forced at world 1
# (1-rank RCCL group, buckets, comm stream, bucket timing recorded).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6models
mkdir -p $O
for m in llama3-8b resnet50; do
for f in "" "--force-ddp"; do
tag=$m${f:+_forceddp}
timeout -k 10 600 python bench.py --model $m --steps 20 --warmup 5 --no-latency $f > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }
python -c "import json; d=json.load(open('$O/$tag.json')); g=d['config'].get('grad_allreduce', {}); print('$tag', d['value'], d['ms_per_step'], d['config'].get('mfu'), g.get('xgmi_tune_s'), g.get('xgmi_timed_buckets'), g.get('buckets'))"
done
done
