#!/bin/bash
# NGP / container GPU tests, then the NGP expert and container bench lines
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ngp.py tests/test_gpu_moe.py tests/test_gpu_occ.py > gpurun_out/t_ngp.log 2>&1 || { tail -40 gpurun_out/t_ngp.log; exit 1; }
tail -1 gpurun_out/t_ngp.log
timeout -k 10 300 python tools/bench_ngp.py --no-cpu-baseline > gpurun_out/bn.log 2>&1 || { tail -30 gpurun_out/bn.log; exit 1; }
tail -1 gpurun_out/bn.log | cut -c1-1500
timeout -k 10 300 python tools/bench_container.py --no-cpu-baseline > gpurun_out/bc.log 2>&1 || { tail -30 gpurun_out/bc.log; exit 1; }
tail -1 gpurun_out/bc.log | cut -c1-1500
