#!/bin/bash
# Round 5, call 13: two 4-wave workgroups per CU (each SIMD: one wave of each) for the split forward (nw4), the split
# input gradient (dg4), and both — one workgroup's epilogue under the other's MFMAs; parity on nw4dg4, then C2 A/B.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
NERF_AMD_LIB=exp/nw4dg4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_split_gemm.py tests/test_gpu_c2_backward.py -m gpu -q \
  --timeout 240 --timeout-method thread > $O/pytest_nw4dg4.log 2>&1; rc=$?; tail -2 $O/pytest_nw4dg4.log
[ $rc -gt 1 ] && exit 1
VARIANTS="x6base nw4 dg4 nw4dg4" ROUNDS=2 timeout -k 10 1000 bash tools/ab_x6.sh
