#!/bin/bash
# One GPU-box session: build check, gpu parity tests, smoke, bench, rocprof kernel stats.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
STEP=${1:-all}
if [[ $STEP == all || $STEP == test ]]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -30 gpurun_out/pytest_gpu.log; [[ $rc -ne 0 ]] && exit $rc
  timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
  cat gpurun_out/smoke.log
fi
if [[ $STEP == all || $STEP == bench ]]; then
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
  tail -3 gpurun_out/bench.log
fi
if [[ $STEP == all || $STEP == prof ]]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --train-views 8 > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
  tail -2 gpurun_out/prof.log
  find gpurun_out/prof -name "*kernel_stats.csv" | head -3
fi
