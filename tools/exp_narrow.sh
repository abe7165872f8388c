#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bf16.py > gpurun_out/t_bf16.log 2>&1 || { tail -40 gpurun_out/t_bf16.log; exit 1; }
tail -1 gpurun_out/t_bf16.log
for m in 1 2; do
  NERF_BF16_NARROW_MUL=$m timeout -k 10 120 python tools/bench_mlp.py --precision bf16 > gpurun_out/nm$m.log 2>&1 || { tail -20 gpurun_out/nm$m.log; exit 1; }
  NERF_BF16_NARROW_MUL=$m timeout -k 10 300 python bench.py --precision bf16 --no-cpu-baseline --no-psnr > gpurun_out/bnm$m.log 2>&1 || { tail -20 gpurun_out/bnm$m.log; exit 1; }
  echo "mul=$m mlp: $(tail -1 gpurun_out/nm$m.log | cut -c1-200) bench: $(tail -1 gpurun_out/bnm$m.log | cut -c100-190)"
done
bash tools/prof_mlp.sh
