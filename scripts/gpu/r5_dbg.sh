#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PTO_XGMI_TIMEOUT_MS=2000
for m in twinrun; do
  timeout -k 10 150 python tools/probes/race_bisect.py $m 2>&1 | grep -v Gloo | tail -3 || { echo "$m rc=$?"; exit 1; }
done
