#!/bin/bash
# F12 / F3 / F4dx phase stamps (probe build of the shipped sources).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6_f3
mkdir -p $O
timeout -k 10 300 python tools/bwd_phases_probe.py --fwd --reps 30 > $O/fwd_phases.txt 2>&1 || { tail -20 $O/fwd_phases.txt; exit 1; }
grep -v amdgpu.ids $O/fwd_phases.txt | head -5
