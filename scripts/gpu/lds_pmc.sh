#!/bin/bash
# LDS counters of the MNIST step kernels per env setting:
#   lds_pmc.sh "PTO_DETERMINISTIC=0" "PTO_DETERMINISTIC=1" ...
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lds
cd /tmp
i=0
for setting in "$@"; do
  i=$((i+1))
  env $setting true
  rm -rf "$R/gpurun_out/lds/pmc_$i"
  ( export $setting; timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES --kernel-trace -d "$R/gpurun_out/lds/pmc_$i" -o run -- python3 "$R/bench.py" --steps 20 --warmup 4 --no-latency > "$R/gpurun_out/lds/pmc_$i.log" 2>&1 ) || { tail -20 "$R/gpurun_out/lds/pmc_$i.log"; exit 1; }
  echo "== $setting"
  python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/lds/pmc_$i" --filter k_
  rm -rf "$R/gpurun_out/lds/pmc_$i"
done
