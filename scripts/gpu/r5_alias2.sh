#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5r
mkdir -p $O
for cfg in "8 64" "256 224"; do
PYTHONPATH=. timeout -k 10 300 python tools/probes/graph_alias_probe.py $cfg > $O/alias.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/alias.txt | tail -8
[ $rc -le 1 ] || exit 1
done
