#!/bin/bash
# Container step anatomy (kernel trace): eager and graph-mode, busy vs wall per step (tools/cont_timeline.py).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06/$1; mkdir -p $O; export TMPDIR=/tmp
for mode in eager graph; do
  F="--no-graph"; [ $mode = graph ] && F="--graph"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$mode -o run --output-format csv -- python3 tools/bench_container.py --no-cpu-baseline --steps 24 --warmup 40 $F > $O/prof_$mode.log 2>&1 || { tail -20 $O/prof_$mode.log; exit 1; }
  python3 tools/cont_timeline.py $O/prof_$mode/run_kernel_trace.csv 30 24 > $O/step_$mode.txt 2>&1 || true
  rm -f $O/prof_$mode/run_kernel_trace.csv
  echo "== $mode"; head -3 $O/step_$mode.txt; tail -2 $O/step_$mode.txt
done
