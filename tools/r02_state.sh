#!/bin/bash
# State check: whole -m gpu suite, smoke, fp32 + bf16 bench lines, rocprof kernel stats of the bf16 bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/t_all.log 2>&1 || { tail -40 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --precision bf16 --no-cpu-baseline --no-psnr > gpurun_out/b_bf16.log 2>&1 || { tail -30 gpurun_out/b_bf16.log; exit 1; }
tail -1 gpurun_out/b_bf16.log | cut -c1-1500
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bf16 -o run --output-format csv -- python3 bench.py --precision bf16 --steps 20 --warmup 5 --no-cpu-baseline --no-psnr --no-dropin > gpurun_out/prof_bf16.log 2>&1 || { tail -20 gpurun_out/prof_bf16.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_bf16/run_kernel_stats.csv 25 > gpurun_out/prof_bf16_summary.txt 2>&1
head -40 gpurun_out/prof_bf16_summary.txt
