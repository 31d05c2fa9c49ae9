#!/bin/bash
# LDS counters of k_bwd_all per role (tools/bwd_roles_probe.py --pmc-mask;
# the probe .so is built on the CPU host beforehand), then of the whole step.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cd /tmp
CTR="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
for m in ${MASKS:-4 8 16 3}; do
  timeout -s KILL 90 rocprofv3 --pmc $CTR --kernel-trace -d "/tmp/roles_$m" -o run -- python3 "$R/tools/bwd_roles_probe.py" --pmc-mask $m > "$R/gpurun_out/roles_pmc_$m.log" 2>&1 || { tail -20 "$R/gpurun_out/roles_pmc_$m.log"; exit 1; }
  echo "== role mask $m"
  python3 "$R/tools/pmc_summary.py" "/tmp/roles_$m" --filter k_bwd_all --skip 3
done
timeout -s KILL 90 rocprofv3 --pmc $CTR --kernel-trace -d /tmp/step_lds -o run -- python3 "$R/bench.py" --steps 20 --warmup 4 --no-latency > "$R/gpurun_out/step_lds.log" 2>&1 || { tail -20 "$R/gpurun_out/step_lds.log"; exit 1; }
echo "== step"
python3 "$R/tools/pmc_summary.py" /tmp/step_lds --filter k_
