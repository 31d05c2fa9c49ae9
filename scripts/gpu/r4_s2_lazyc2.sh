#!/bin/bash
# lazy conv2.weight update (PTO_LAZY_C2): numerics tests (kernels, graphs,
# one-epoch parity, DDP), then bench A/B at 2000 steps and the driver's
# command, kernel stats of both.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lz
timeout -k 10 700 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py tests/test_parity_long_gpu.py tests/test_ddp_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/lz/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/lz/pytest.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/lz/pytest.log | head -20; exit 1; }
for v in 1 0 1 0; do
  PTO_LAZY_C2=$v timeout -k 10 200 python bench.py --no-latency > gpurun_out/lz/b2000_$v.json 2> gpurun_out/lz/b2000_$v.err || { tail -5 gpurun_out/lz/b2000_$v.err; exit 1; }
  echo "lazy=$v 2000: $(cut -c1-150 gpurun_out/lz/b2000_$v.json)"
done
for v in 1 0 1; do
  PTO_LAZY_C2=$v timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-latency > gpurun_out/lz/bdrv_$v.json 2> gpurun_out/lz/bdrv_$v.err || { tail -5 gpurun_out/lz/bdrv_$v.err; exit 1; }
  echo "lazy=$v drv: $(cut -c1-150 gpurun_out/lz/bdrv_$v.json)"
done
cd /tmp
for v in 1 0; do
  rm -rf /tmp/kst_$v
  PTO_LAZY_C2=$v timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kst_$v -o run -- python3 "$R/bench.py" --steps 400 --warmup 40 --no-latency > "$R/gpurun_out/lz/prof_$v.log" 2>&1 || exit 1
  f=$(find /tmp/kst_$v -name "*kernel_stats.csv" | head -1)
  echo "== lazy=$v"; python3 "$R/tools/kstats_table.py" "$f" | head -6 | tee "$R/gpurun_out/lz/kstats_$v.txt"
done
