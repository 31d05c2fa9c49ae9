#!/bin/bash
# Round 2 check: config-2 rehearsal e2e tests, bench (20 / 2000 steps),
# rocprofv3 kernel stats + two SQ counter passes of the shipped MNIST step.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_bench20.log 2>&1
tail -1 gpurun_out/r2_bench20.log
timeout -k 10 200 python bench.py --no-latency > gpurun_out/r2_bench2000.log 2>&1
tail -1 gpurun_out/r2_bench2000.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r2_pytest_gpu.log 2>&1 || { tail -60 gpurun_out/r2_pytest_gpu.log; exit 1; }
tail -8 gpurun_out/r2_pytest_gpu.log
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r2_prof" -o run -- python3 "$R/bench.py" --steps 50 --warmup 10 --no-latency > "$R/gpurun_out/r2_prof.log" 2>&1
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d "$R/gpurun_out/r2_pmc_$i" -o run -- python3 "$R/bench.py" --steps 20 --warmup 4 --no-latency > "$R/gpurun_out/r2_pmc_$i.log" 2>&1 || { tail -20 "$R/gpurun_out/r2_pmc_$i.log"; exit 1; }
done
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/r2_pmc_1" "$R/gpurun_out/r2_pmc_2" --filter k_ > "$R/gpurun_out/r2_pmc_summary.txt"
cat "$R/gpurun_out/r2_pmc_summary.txt"
