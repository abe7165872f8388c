#!/bin/bash
# fused bf16 backward: bitwise parity vs the layered backward, the bf16 tests, MLP timing A/B, bf16 bench line
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bf16.py > gpurun_out/t_bf16.log 2>&1 || { tail -40 gpurun_out/t_bf16.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/t_bf16.log | tail -15
for m in 0 1; do
  NERF_BF16_FUSED_BWD=$m timeout -k 10 120 python tools/bench_mlp.py --precision bf16 > gpurun_out/mlp_bwd$m.log 2>&1 || { tail -20 gpurun_out/mlp_bwd$m.log; exit 1; }
  echo "fused_bwd=$m $(tail -1 gpurun_out/mlp_bwd$m.log)"
done
timeout -k 10 300 python bench.py --precision bf16 --no-cpu-baseline --no-psnr > gpurun_out/b_bf16.log 2>&1 || { tail -30 gpurun_out/b_bf16.log; exit 1; }
tail -1 gpurun_out/b_bf16.log | cut -c1-400
