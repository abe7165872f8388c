#!/bin/bash
# Round 5, call 14: the packed fp16 epilogue of the fused forward + four row parts in the fp32 colour / head backward:
# parity (fp16, drop-in, fp32 MLP, C2 backward, edges), the AMP A/B, then C2 A/B of the tail parts (2 / 4 / 8).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp16.py tests/test_gpu_dropin.py tests/test_gpu_parity.py tests/test_gpu_c2_backward.py \
  tests/test_gpu_edges.py tests/test_gpu_split_gemm.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_c14.log 2>&1; rc=$?
tail -3 $O/pytest_c14.log; grep -E "FAIL|Error" $O/pytest_c14.log | head -10
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python3 tools/amp_kernels_ab.py > $O/amp_ab_c14.log 2>&1 || { tail -20 $O/amp_ab_c14.log; exit 1; }
grep -E "^(fp16|bf16)" $O/amp_ab_c14.log
VARIANTS="tq2 tq4 tq8" ROUNDS=2 timeout -k 10 700 bash tools/ab_x6.sh
