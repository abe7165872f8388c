#!/bin/bash
# A/B of the guard-free weight-gradient slab loop (NERF_X6W_WG_NOGUARD) against HEAD: tests, then alternating C2 rounds.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/wg; export TMPDIR=/tmp
NERF_AMD_LIB=exp/wgng.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_split_gemm.py tests/test_gpu_parity.py tests/test_gpu_c2_backward.py > gpurun_out/wg/t.log 2>&1 || { tail -30 gpurun_out/wg/t.log; exit 1; }
echo "wgng: $(tail -1 gpurun_out/wg/t.log)"
VARIANTS="base6 wgng" ROUNDS=${ROUNDS:-3} tools/ab_x6.sh
