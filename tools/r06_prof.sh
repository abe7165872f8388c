#!/bin/bash
# Round-6 profiles: the container step (bench line + rocprof kernel trace -> per-step kernel time vs wall), and the
# C2 / C3 engine steps (kernel stats + one step's timeline).  Outputs under gpurun_out/r06/$1.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06/$1; mkdir -p $O; export TMPDIR=/tmp
if [ -z "$SKIP_CONT" ]; then
timeout -k 10 300 python tools/bench_container.py --no-cpu-baseline > $O/bc.log 2>&1 || { tail -30 $O/bc.log; exit 1; }
tail -1 $O/bc.log | cut -c1-1500
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cont -o run --output-format csv -- python3 tools/bench_container.py --no-cpu-baseline --steps 10 --warmup 34 > $O/prof_cont.log 2>&1 || { tail -20 $O/prof_cont.log; exit 1; }
python3 tools/prof_summary.py $O/prof_cont/run_kernel_stats.csv 40 > $O/prof_cont_summary.txt 2>&1
python3 tools/cont_timeline.py $O/prof_cont/run_kernel_trace.csv > $O/step_cont.txt 2>&1 || true
tail -5 $O/step_cont.txt
fi
[ -n "$SKIP_ENGINE" ] && exit 0
for P in ${PRECS:-bf16 fp32}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$P -o run --output-format csv -- \
    python3 bench.py --precision $P --steps 20 --warmup 5 --no-cpu-baseline --no-psnr --no-dropin --no-other-precision --no-native-ref --no-ngp --no-container --no-llff --no-sweep \
    > $O/prof_$P.log 2>&1 || { tail -20 $O/prof_$P.log; exit 1; }
  python3 tools/prof_summary.py $O/prof_$P/run_kernel_stats.csv 28 3 > $O/prof_${P}_summary.txt 2>&1
  python3 tools/step_timeline.py $O/prof_$P/run_kernel_trace.csv > $O/step_${P}.txt 2>&1 || true
  rm -f $O/prof_$P/run_kernel_trace.csv
  echo "prof $P: $(tail -1 $O/prof_$P.log | cut -c1-200)"
done
