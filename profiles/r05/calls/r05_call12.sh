#!/bin/bash
# Round 5, call 12: the forward split GEMM on 12 32-row waves (three per SIMD) vs the default 8 64-row waves:
# split-GEMM parity tests on the variant build, then the C2 A/B (tools/ab_x6.sh, alternating builds).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
NERF_AMD_LIB=exp/w12.so timeout -k 10 300 python -u -m pytest tests/test_gpu_split_gemm.py tests/test_gpu_c2_backward.py -m gpu -q \
  --timeout 240 --timeout-method thread > $O/pytest_w12.log 2>&1; rc=$?; tail -2 $O/pytest_w12.log
[ $rc -gt 1 ] && exit 1
VARIANTS="x6base w12" ROUNDS=3 timeout -k 10 900 bash tools/ab_x6.sh
