#!/bin/bash
# Round-2 artifacts of the §8f rows: NGP expert + container bench lines, rocprof kernel stats and one-step timeline of
# each, per-step container times (occupancy-update steps).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/art && export TMPDIR=/tmp
O=gpurun_out/art
timeout -k 10 300 python tools/bench_ngp.py > $O/bench_ngp.log 2>&1 || { tail -30 $O/bench_ngp.log; exit 1; }
tail -1 $O/bench_ngp.log | cut -c1-300
timeout -k 10 300 python tools/bench_container.py > $O/bench_container.log 2>&1 || { tail -30 $O/bench_container.log; exit 1; }
tail -1 $O/bench_container.log | cut -c1-300
timeout -k 10 300 python tools/container_steps.py > $O/container_steps.log 2>&1 || { tail -30 $O/container_steps.log; exit 1; }
tail -2 $O/container_steps.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ngp -o run --output-format csv -- python3 tools/bench_ngp.py --no-cpu-baseline --steps 10 --warmup 3 > $O/prof_ngp.log 2>&1 || { tail -20 $O/prof_ngp.log; exit 1; }
python3 tools/prof_summary.py $O/prof_ngp/run_kernel_stats.csv 25 > $O/prof_ngp_summary.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cont -o run --output-format csv -- python3 tools/bench_container.py --no-cpu-baseline --steps 10 --warmup 34 > $O/prof_cont.log 2>&1 || { tail -20 $O/prof_cont.log; exit 1; }
python3 tools/prof_summary.py $O/prof_cont/run_kernel_stats.csv 30 > $O/prof_cont_summary.txt 2>&1
python3 tools/step_timeline.py $O/prof_cont/run_kernel_trace.csv > $O/step_cont.txt 2>&1
tail -1 $O/step_cont.txt
