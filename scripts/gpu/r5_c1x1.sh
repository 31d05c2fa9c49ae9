#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5r
mkdir -p $O
timeout -k 10 400 python tools/conv1x1_bench.py > $O/c1x1.jsonl 2> $O/c1x1.err || { tail -20 $O/c1x1.err; exit 1; }
cat $O/c1x1.jsonl
