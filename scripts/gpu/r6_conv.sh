#!/bin/bash
# Round 6: the 3x3 conv kernel -- numerics tests, per-shape timing against
# MIOpen, then (if correct) the ResNet-50 bench.  Also the rehearsal A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6conv
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_conv3x3_gpu.py -v -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|Error" $O/pytest.log | tail -16
case $rc in 0) ;; 1) tail -40 $O/pytest.log;; *) echo "pytest rc=$rc"; exit $rc;; esac
timeout -k 10 300 python -u tools/conv3x3_bench.py --variants 64:1,32:3,32:4,32:5 > $O/bench.jsonl 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.jsonl
exit $rc
