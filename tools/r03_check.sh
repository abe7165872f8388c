#!/bin/bash
# Round-3 check on one GPU box: the changed / new GPU tests, the default bench line, a 2-rank gloo rehearsal.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TESTS:-"tests/test_gpu_dropin.py tests/test_gpu_bf16.py tests/test_gpu_ngp.py tests/test_gpu_configs.py tests/test_gpu_meta.py tests/test_gpu_dp.py"}
timeout -k 10 600 python -u -m pytest $T -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_r03.log 2>&1 || { tail -40 gpurun_out/pytest_r03.log; exit 1; }
tail -3 gpurun_out/pytest_r03.log
timeout -k 10 500 python bench.py > gpurun_out/bench_r03.log 2>&1 || { tail -30 gpurun_out/bench_r03.log; exit 1; }
tail -1 gpurun_out/bench_r03.log | cut -c1-600
timeout -k 10 200 python bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --no-psnr --no-cpu-baseline > gpurun_out/bench_gloo2.log 2>&1 || { tail -30 gpurun_out/bench_gloo2.log; exit 1; }
tail -1 gpurun_out/bench_gloo2.log | cut -c1-300
