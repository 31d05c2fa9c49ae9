#!/bin/bash
# ResNet-50 bench run-to-run spread: independent MIOpen finds vs a shared find DB.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5v
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 --no-latency > $O/fresh$i.json 2> $O/fresh$i.err || { tail -20 $O/fresh$i.err; exit 1; }
  python -c "import json;d=json.load(open('$O/fresh$i.json'));print('fresh',$i,d['value'],d['ms_per_step'])"
  rm -rf ~/.config/miopen ~/.cache/miopen 2>/dev/null
done
export MIOPEN_USER_DB_PATH=$PWD/$O/udb
mkdir -p $MIOPEN_USER_DB_PATH
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 --no-latency > $O/db$i.json 2> $O/db$i.err || { tail -20 $O/db$i.err; exit 1; }
  python -c "import json;d=json.load(open('$O/db$i.json'));print('shared-db',$i,d['value'],d['ms_per_step'])"
done
ls -la $MIOPEN_USER_DB_PATH
