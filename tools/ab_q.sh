#!/bin/bash
# 16x16x32 split NT forward (exp/x6q.so, built -DNERF_X6_Q) vs 32x32x16 (exp/x6w.so): accuracy tests, then C2 A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out && export TMPDIR=/tmp
for v in ${QVARIANTS:-x6q}; do
NERF_AMD_LIB=exp/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_split_gemm.py -x -v -s --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_$v.log 2>&1 || { grep -E "Error|assert|FAIL" gpurun_out/pytest_$v.log | tail -20; exit 1; }
tail -1 gpurun_out/pytest_$v.log
done
VARIANTS="${VARIANTS:-x6w x6q}" ROUNDS=${ROUNDS:-2} BENCH_EXTRA="--no-native-ref" bash tools/ab_x6.sh
