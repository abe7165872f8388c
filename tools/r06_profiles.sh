#!/bin/bash
# Round-6 profiles: rocprof kernel stats + one step's timeline of the C2 (fp32) and C3 (bf16) bench legs, PMC HBM
# traffic (FETCH_SIZE / WRITE_SIZE passes) of the fine-net kernels for both precisions, and the split GEMMs' wave-cycle
# / MFMA-busy / LDS-conflict pass.  Outputs under gpurun_out/r06/$1.  (The full-bench PMC pass of round 5 is not rerun.)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06/$1; mkdir -p $O; export TMPDIR=/tmp
if [ -z "$SKIP_PROF" ]; then
for P in fp32 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$P -o run --output-format csv -- \
    python3 bench.py --precision $P --steps 20 --warmup 5 --no-cpu-baseline --no-psnr --no-dropin --no-other-precision --no-native-ref --no-ngp --no-container --no-llff --no-sweep \
    > $O/prof_$P.log 2>&1 || { tail -20 $O/prof_$P.log; exit 1; }
  python3 tools/prof_summary.py $O/prof_$P/run_kernel_stats.csv 28 3 > $O/prof_${P}_summary.txt 2>&1
  python3 tools/step_timeline.py $O/prof_$P/run_kernel_trace.csv mid > $O/step_${P}.txt 2>&1 || true
  python3 tools/step_timeline.py $O/prof_$P/run_kernel_trace.csv last > $O/step_${P}_events.txt 2>&1 || true
  rm -f $O/prof_$P/run_kernel_trace.csv
  echo "prof $P: $(tail -1 $O/prof_$P.log | cut -c1-160)"
done
fi
[ -n "$STOP_AFTER_PROF" ] && exit 0
export LEG_ARGS="--no-llff --no-sweep"
PMC_OUT=$O/pmc_fp32 PMC_BENCH_ARGS="--no-dropin --no-other-precision --no-native-ref" bash tools/pmc_traffic.sh > $O/pmc_fp32.txt 2>&1 || { tail -20 $O/pmc_fp32.txt; exit 1; }
PMC_OUT=$O/pmc_bf16 PMC_PRECISION=bf16fused PMC_BENCH_ARGS="--precision bf16 --no-dropin --no-other-precision" bash tools/pmc_traffic.sh > $O/pmc_bf16.txt 2>&1 || { tail -20 $O/pmc_bf16.txt; exit 1; }
tail -n 2 $O/pmc_fp32.txt; tail -n 2 $O/pmc_bf16.txt
find $O/pmc_fp32 $O/pmc_bf16 -name "*.csv" -size +4M -delete 2>/dev/null
VARIANTS=split bash tools/pmc_split.sh > $O/pmc_split.txt 2>&1 || { tail -20 $O/pmc_split.txt; exit 1; }
cp gpurun_out/pmc_split_split/summary.txt $O/pmc_split_summary.txt 2>/dev/null
tail -n 4 $O/pmc_split.txt | cut -c1-200
find gpurun_out/pmc_split_split -name "*.csv" -size +4M -delete 2>/dev/null
