#!/bin/bash
# quick GPU check of the fp32 headline path: MLP / render parity tests, bench, rocprof kernel stats
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/tq.log 2>&1 || { tail -40 gpurun_out/tq.log; exit 1; }
tail -n 1 gpurun_out/tq.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-psnr ${BENCH_ARGS} > gpurun_out/bq.log 2>&1 || { tail -20 gpurun_out/bq.log; exit 1; }
tail -n 1 gpurun_out/bq.log | cut -c1-900
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profq -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-psnr ${BENCH_ARGS} > gpurun_out/profq.log 2>&1 || { tail -20 gpurun_out/profq.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/profq/run_kernel_stats.csv 14 > gpurun_out/profq_summary.txt 2>&1; python3 tools/pergrid.py gpurun_out/profq/run_kernel_trace.csv
