#!/bin/bash
# bf16 GPU tests + the C3 bench line (+ optional extra bench args in BENCH_ARGS)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bf16.py tests/test_gpu_dp.py > gpurun_out/t_bf16.log 2>&1 || { tail -40 gpurun_out/t_bf16.log; exit 1; }
tail -1 gpurun_out/t_bf16.log
timeout -k 10 300 python bench.py --precision bf16 --no-cpu-baseline --no-psnr $BENCH_ARGS > gpurun_out/b_bf16.log 2>&1 || { tail -30 gpurun_out/b_bf16.log; exit 1; }
tail -1 gpurun_out/b_bf16.log | cut -c1-300
