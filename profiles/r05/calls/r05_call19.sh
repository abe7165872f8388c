#!/bin/bash
# Round 5, call 19: the dot-form split in the forward only (the new default) against the round-4 split: parity on the
# default library, then the C2 A/B (loss bitwise the same).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_split_gemm.py tests/test_gpu_c2_backward.py tests/test_gpu_parity.py -m gpu -q \
  --timeout 240 --timeout-method thread > $O/pytest_dot2fwd.log 2>&1; rc=$?; tail -2 $O/pytest_dot2fwd.log
[ $rc -ne 0 ] && exit 1
VARIANTS="x6base dot2fwd" ROUNDS=3 timeout -k 10 800 bash tools/ab_x6.sh
