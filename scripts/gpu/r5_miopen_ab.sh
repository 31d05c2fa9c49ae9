#!/bin/bash
# ResNet-50: MIOpen's asm implicit-GEMM NHWC backward solvers (which zero
# their outputs with SubTensorOp kernels first) on / off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5m2
mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 400 python bench.py --model resnet50 --steps 20 --warmup 5 --no-latency > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'])"
}
case "${1:-bwd}" in
bwd)
run base PTO_X=1 && \
run nobwd MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 && \
run nowrw MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 && \
run noboth MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 && \
run base2 PTO_X=1 ;;
fwd)  # the stem's forward solver (asm implicit GEMM + a zero-fill of its output) vs the next-best
run base PTO_X=1 && \
run nofwd MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0 && \
run base2 PTO_X=1 && \
run nofwd2 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0 ;;
esac
