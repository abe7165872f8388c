#!/bin/bash
# bench line + rocprof kernel trace/stats of the same bench command; PREC=fp32|bf16, extra args in BENCH_ARGS
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out && export TMPDIR=/tmp
P=${PREC:-bf16}
timeout -k 10 300 python bench.py --precision $P --no-cpu-baseline --no-psnr $BENCH_ARGS > gpurun_out/b_$P.log 2>&1 || { tail -30 gpurun_out/b_$P.log; exit 1; }
tail -1 gpurun_out/b_$P.log | cut -c1-3000
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$P -o run --output-format csv -- python3 bench.py --precision $P --steps 20 --warmup 5 --no-cpu-baseline --no-psnr --no-dropin --no-ngp --no-container $LEG_ARGS $BENCH_ARGS > gpurun_out/prof_$P.log 2>&1 || { tail -20 gpurun_out/prof_$P.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_$P/run_kernel_stats.csv 25 > gpurun_out/prof_${P}_summary.txt 2>&1
python3 tools/step_timeline.py gpurun_out/prof_$P/run_kernel_trace.csv > gpurun_out/step_${P}.txt 2>&1
head -30 gpurun_out/prof_${P}_summary.txt
