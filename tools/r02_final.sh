#!/bin/bash
# Round-2 artifacts at HEAD (after the 16x16x4 trunk GEMMs): whole -m gpu suite, smoke, fp32 bench (engine + drop-in
# + CPU baseline), bf16 bench, rocprof kernel stats + step timelines of both, fp32 PMC HBM traffic.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/fin && export TMPDIR=/tmp
O=gpurun_out/fin
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu_all.log 2>&1 || { tail -40 $O/pytest_gpu_all.log; exit 1; }
tail -1 $O/pytest_gpu_all.log
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_fp32.log 2>&1 || { tail -30 $O/bench_fp32.log; exit 1; }
tail -1 $O/bench_fp32.log | cut -c1-300
timeout -k 10 300 python bench.py --precision bf16 --no-cpu-baseline > $O/bench_bf16.log 2>&1 || { tail -30 $O/bench_bf16.log; exit 1; }
tail -1 $O/bench_bf16.log | cut -c1-300
for P in fp32 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$P -o run --output-format csv -- python3 bench.py --precision $P --steps 20 --warmup 5 --no-cpu-baseline --no-psnr --no-dropin > $O/prof_$P.log 2>&1 || { tail -20 $O/prof_$P.log; exit 1; }
  python3 tools/prof_summary.py $O/prof_$P/run_kernel_stats.csv 25 > $O/prof_${P}_summary.txt 2>&1
  python3 tools/step_timeline.py $O/prof_$P/run_kernel_trace.csv > $O/step_${P}.txt 2>&1
done
PMC_OUT=$O/pmc_fp32 PMC_BENCH_ARGS="--no-dropin" bash tools/pmc_traffic.sh > $O/pmc_fp32.log 2>&1 || { tail -20 $O/pmc_fp32.log; exit 1; }
tail -1 $O/pmc_fp32.log
