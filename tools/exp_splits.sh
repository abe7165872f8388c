#!/bin/bash
# bf16 split-count A/B: MLP timing and the bf16 bench line per NERF_BF16_MAX_SPLITS
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bf16.py > gpurun_out/t_bf16.log 2>&1 || { tail -40 gpurun_out/t_bf16.log; exit 1; }
tail -1 gpurun_out/t_bf16.log
for sp in 128 256; do
  NERF_BF16_MAX_SPLITS=$sp timeout -k 10 120 python tools/bench_mlp.py --precision bf16 > gpurun_out/sp$sp.log 2>&1 || { tail -20 gpurun_out/sp$sp.log; exit 1; }
  NERF_BF16_MAX_SPLITS=$sp timeout -k 10 300 python bench.py --precision bf16 --no-cpu-baseline --no-psnr > gpurun_out/bsp$sp.log 2>&1 || { tail -20 gpurun_out/bsp$sp.log; exit 1; }
  echo "splits=$sp mlp: $(tail -1 gpurun_out/sp$sp.log) bench: $(tail -1 gpurun_out/bsp$sp.log | cut -c100-200)"
done
