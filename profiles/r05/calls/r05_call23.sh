#!/bin/bash
# Round 5, call 23: the split forward on 256 x 256 tiles (32 x 256 waves; -DNERF_X6_FWD_TN8) vs the default 512 x 128:
# parity on the variant, bitwise fp32 outputs of the two builds, then the C2 A/B.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
NERF_AMD_LIB=exp/tn8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_split_gemm.py tests/test_gpu_c2_backward.py tests/test_gpu_parity.py -m gpu -q \
  --timeout 240 --timeout-method thread > $O/pytest_tn8.log 2>&1; rc=$?; tail -2 $O/pytest_tn8.log; grep -E "FAIL|Error" $O/pytest_tn8.log | head -5
[ $rc -ne 0 ] && exit 1
NERF_AMD_LIB=exp/tn8.so timeout -k 10 120 python tools/lib_outputs.py --precision fp32 --out $O/tn8.pt > $O/lo_tn8.log 2>&1 || { tail $O/lo_tn8.log; exit 1; }
NERF_AMD_LIB=exp/x6base.so timeout -k 10 120 python tools/lib_outputs.py --precision fp32 --out $O/base.pt > $O/lo_base.log 2>&1 || { tail $O/lo_base.log; exit 1; }
python tools/lib_outputs.py --compare $O/tn8.pt $O/base.pt; rm -f $O/tn8.pt $O/base.pt
VARIANTS="x6base tn8" ROUNDS=3 timeout -k 10 800 bash tools/ab_x6.sh
