#!/bin/bash
# data-parallel GPU tests (world 2 over gloo on one GPU)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dp.py > gpurun_out/t_dp.log 2>&1 || { tail -40 gpurun_out/t_dp.log; exit 1; }
tail -5 gpurun_out/t_dp.log
