#!/bin/bash
# Round 5, call 18: split residuals by v_dot2c_f32_bf16 (-DNERF_X6_DOT2SPLIT): split-GEMM parity tests on the variant,
# then the C2 A/B against the default (the loss must be bitwise the same: the pieces are).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
NERF_AMD_LIB=exp/dot2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_split_gemm.py tests/test_gpu_c2_backward.py tests/test_gpu_parity.py -m gpu -q \
  --timeout 240 --timeout-method thread > $O/pytest_dot2.log 2>&1; rc=$?; tail -3 $O/pytest_dot2.log; grep -E "FAIL|Error" $O/pytest_dot2.log | head
[ $rc -ne 0 ] && exit 1
VARIANTS="x6base dot2" ROUNDS=3 timeout -k 10 800 bash tools/ab_x6.sh
