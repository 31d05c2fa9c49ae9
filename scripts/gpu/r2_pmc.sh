#!/bin/bash
# rocprofv3 kernel stats + two SQ counter passes of the shipped MNIST step
# (raw profiler output under /tmp: only the summary goes to gpurun_out)
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
TAG=${1:-r2}
mkdir -p gpurun_out
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "/tmp/${TAG}_prof" -o run -- python3 "$R/bench.py" --steps 50 --warmup 10 --no-latency > "$R/gpurun_out/${TAG}_prof.log" 2>&1
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d "/tmp/${TAG}_pmc_$i" -o run -- python3 "$R/bench.py" --steps 20 --warmup 4 --no-latency > "$R/gpurun_out/${TAG}_pmc_$i.log" 2>&1 || { tail -20 "$R/gpurun_out/${TAG}_pmc_$i.log"; exit 1; }
done
python3 "$R/tools/pmc_summary.py" "/tmp/${TAG}_pmc_1" "/tmp/${TAG}_pmc_2" --filter k_ > "$R/gpurun_out/${TAG}_pmc_summary.txt"
cat "$R/gpurun_out/${TAG}_pmc_summary.txt"
