#!/bin/bash
# where the training image's time to its first step goes: cProfile of a
# fresh `python -m pytorch_operator_1_amd.train.mnist` (world 1, GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/st
timeout -k 10 300 python -m cProfile -o gpurun_out/st/image.prof -m pytorch_operator_1_amd.train.mnist --max-steps 20 --log-interval 10 --dir "" > gpurun_out/st/image.log 2>&1 || { tail -20 gpurun_out/st/image.log; exit 1; }
python - <<'PY' > gpurun_out/st/image_prof.txt
import pstats
s = pstats.Stats("gpurun_out/st/image.prof")
s.sort_stats("cumulative").print_stats(60)
s.sort_stats("tottime").print_stats(25)
PY
head -120 gpurun_out/st/image_prof.txt | tail -90
