#!/bin/bash
# submit -> first-step latency on the GPU (zygote on/off) + MNIST step PMC counters
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
timeout -k 10 400 python tools/first_step_latency.py --gpu --runs 2 > gpurun_out/latency_gpu.jsonl 2> gpurun_out/latency_gpu.err || { tail -30 gpurun_out/latency_gpu.err; exit 1; }
cat gpurun_out/latency_gpu.jsonl
cd /tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d "$R/gpurun_out/pmc_mnist_$i" -o run -- python3 "$R/bench.py" --steps 20 --warmup 4 > "$R/gpurun_out/pmc_mnist_$i.log" 2>&1 || { tail -20 "$R/gpurun_out/pmc_mnist_$i.log"; exit 1; }
done
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/pmc_mnist_1" "$R/gpurun_out/pmc_mnist_2" --filter k_ > "$R/gpurun_out/pmc_mnist_summary.txt"
cat "$R/gpurun_out/pmc_mnist_summary.txt"
