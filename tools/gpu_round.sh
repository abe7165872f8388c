#!/bin/bash
# One GPU-box session: gpu parity tests, smoke, bench, rocprof kernel stats of the same bench command,
# PMC HBM traffic.  Usage: tools/gpu_round.sh [all|test|bench|prof|pmc]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
STEP=${1:-all}
BENCH_ARGS=${BENCH_ARGS:-"--steps 20 --warmup 5"}
if [[ $STEP == all || $STEP == test ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -30 gpurun_out/pytest_gpu.log; [[ $rc -ne 0 ]] && exit $rc
  timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
  cat gpurun_out/smoke.log
fi
if [[ $STEP == all || $STEP == bench ]]; then
  timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
  tail -1 gpurun_out/bench.log
fi
if [[ $STEP == all || $STEP == prof ]]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
    python3 bench.py $BENCH_ARGS --no-cpu-baseline --no-psnr > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
  python3 tools/prof_summary.py gpurun_out/prof/run_kernel_stats.csv 25 > gpurun_out/prof_summary.txt 2>&1
  tail -1 gpurun_out/prof.log | cut -c1-200
fi
if [[ $STEP == all || $STEP == pmc ]]; then
  bash tools/pmc_traffic.sh || exit 1
fi
