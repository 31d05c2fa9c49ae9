#!/bin/bash
# Attention kernels at the Llama-3-8B shape (4 x 4096, 32/8 heads): kernel
# trace + two SQ counter passes (tools/attn_prof.py).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_attention_gpu.py -x -q > gpurun_out/attn_pytest.log 2>&1 || { tail -40 gpurun_out/attn_pytest.log; exit 1; }
tail -1 gpurun_out/attn_pytest.log
cd /tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/attn_trace" -o run -- python3 "$R/tools/attn_prof.py" > "$R/gpurun_out/attn_trace.log" 2>&1 || { tail -20 "$R/gpurun_out/attn_trace.log"; exit 1; }
python3 "$R/tools/rocprof_summary.py" "$R/gpurun_out/attn_trace" --top 8
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  ITERS=1 timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d "$R/gpurun_out/attn_pmc_$i" -o run -- python3 "$R/tools/attn_prof.py" > "$R/gpurun_out/attn_pmc_$i.log" 2>&1 || { tail -20 "$R/gpurun_out/attn_pmc_$i.log"; exit 1; }
done
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/attn_pmc_1" "$R/gpurun_out/attn_pmc_2" --filter attn > "$R/gpurun_out/attn_pmc_summary.txt"
cat "$R/gpurun_out/attn_pmc_summary.txt"
