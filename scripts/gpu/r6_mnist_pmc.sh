#!/bin/bash
# Round 6: the N=1 MNIST step's evidence -- two SQ counter passes over the
# shipped step (bench.py, the driver's path), k_bwd_all's per-role phase
# stamps (mask 31 = all roles, 8 = dgrad alone, 4 = wgrad alone), F12/F4dx
# phases, the role-ablation probe, and the 2000-step steady state.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
O=gpurun_out/r6mnist
mkdir -p $O
timeout -k 10 200 python bench.py --no-latency > $O/bench2000.json 2> $O/bench2000.err || { tail -20 $O/bench2000.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench2000.json')); print('bench 2000 steps', d['value'], d['ms_per_step'])"
timeout -k 10 120 python tools/bwd_phases_probe.py > $O/bwd_phases.txt 2>&1 || { tail -20 $O/bwd_phases.txt; exit 1; }
timeout -k 10 120 python tools/bwd_phases_probe.py --fwd > $O/fwd_phases.txt 2>&1 || { tail -20 $O/fwd_phases.txt; exit 1; }
timeout -k 10 200 python tools/bwd_roles_probe.py > $O/bwd_roles.txt 2>&1 || { tail -20 $O/bwd_roles.txt; exit 1; }
timeout -k 10 100 python tools/dispatch_ramp_probe.py > $O/ramp.txt 2>&1 || { tail -20 $O/ramp.txt; exit 1; }
cat $O/bwd_phases.txt $O/fwd_phases.txt $O/bwd_roles.txt | tail -60
cd /tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d "/tmp/m6_pmc_$i" -o run -- python3 "$R/bench.py" --steps 20 --warmup 4 --no-latency > "$R/$O/pmc_$i.log" 2>&1 || { tail -20 "$R/$O/pmc_$i.log"; exit 1; }
done
python3 "$R/tools/pmc_summary.py" /tmp/m6_pmc_1 /tmp/m6_pmc_2 --filter k_ --skip 3 > "$R/$O/pmc_summary.txt"
cat "$R/$O/pmc_summary.txt"
