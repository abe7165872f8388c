#!/bin/bash
# container + NGP expert bench lines, and a rocprof kernel trace of the container step (GPU busy time per step)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_container.py --no-cpu-baseline > gpurun_out/bc.log 2>&1 || { tail -30 gpurun_out/bc.log; exit 1; }
tail -1 gpurun_out/bc.log | cut -c1-2500
timeout -k 10 300 python tools/bench_ngp.py --no-cpu-baseline > gpurun_out/bn.log 2>&1 || { tail -30 gpurun_out/bn.log; exit 1; }
tail -1 gpurun_out/bn.log | cut -c1-2500
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cont -o run --output-format csv -- python3 tools/bench_container.py --no-cpu-baseline --steps 10 --warmup 34 > gpurun_out/prof_cont.log 2>&1 || { tail -20 gpurun_out/prof_cont.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_cont/run_kernel_stats.csv 30 > gpurun_out/prof_cont_summary.txt 2>&1
python3 tools/step_timeline.py gpurun_out/prof_cont/run_kernel_trace.csv > gpurun_out/step_cont.txt 2>&1
head -40 gpurun_out/prof_cont_summary.txt
tail -3 gpurun_out/step_cont.txt
