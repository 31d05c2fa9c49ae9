#!/bin/bash
# dK/dV producer/consumer issue-priority A/B (PTO_ATTN_DKDV_PRIO 0/1/2), twice each.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for p in 0 1 2 0 1 2; do
  PTO_ATTN_DKDV_PRIO=$p timeout -k 10 120 python tools/attn_ab.py | sed "s/^/prio=$p /" | tee -a gpurun_out/attn_prio.jsonl
done
