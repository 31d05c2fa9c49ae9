#!/bin/bash
# DDP path forced at world 1 (1-rank RCCL group, copy-mode buckets, comm
# stream) vs the plain dp1 step, ResNet-50 and Llama-3-8B, same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5fd
mkdir -p $O
for m in resnet50 llama3-8b; do for f in 0 1; do
extra=""; [ $f = 1 ] && extra="--force-ddp"
timeout -k 10 600 python bench.py --model $m --steps 20 --warmup 5 --no-latency $extra > $O/${m}_ddp$f.json 2> $O/${m}_ddp$f.err || { tail -20 $O/${m}_ddp$f.err; exit 1; }
python -c "import json; d=[json.loads(l) for l in open('$O/${m}_ddp$f.json') if l.startswith('{')][0]; print('$m force_ddp=$f', d['value'], d['ms_per_step'], d['config'].get('parallelism'), d['config'].get('grad_allreduce', {}).get('buckets') if isinstance(d['config'].get('grad_allreduce'), dict) else '')"
done; done
