#!/bin/bash
# Round-2 GPU check: the new parity / config / data-parallel tests, the whole -m gpu suite, the default bench
# (engine + drop-in + CPU baseline) and a 2-rank self-launched bench rehearsal over gloo on the one visible GPU.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out && export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 900 $T tests/test_gpu_edges.py tests/test_gpu_configs.py tests/test_gpu_dp.py > gpurun_out/t_new.log 2>&1 || { tail -60 gpurun_out/t_new.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/t_new.log | tail -30
timeout -k 10 900 $T tests > gpurun_out/t_all.log 2>&1 || { tail -40 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 600 python bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --no-psnr > gpurun_out/bench_g2.log 2>&1 || { tail -30 gpurun_out/bench_g2.log; exit 1; }
tail -1 gpurun_out/bench_g2.log
