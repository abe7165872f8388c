#!/bin/bash
# Round-5 evidence on one GPU box: the default bench line, rocprof kernel stats of the bench command (fp32 and bf16),
# PMC HBM traffic (FETCH_SIZE / WRITE_SIZE passes) and MFMA busy of the bench's kernels.  Outputs under gpurun_out/r05.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
if [ -n "$PMC_ONLY" ] || [ -n "$FULL_PMC_ONLY" ]; then SKIP_TESTS=1; SKIP_BENCH=1; SKIP_PROF=1; fi
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_all.log 2>&1 || { tail -30 $O/pytest_gpu_all.log; exit 1; }
  tail -1 $O/pytest_gpu_all.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 560 python bench.py > $O/bench_default.log 2>&1 || { tail -30 $O/bench_default.log; exit 1; }
  tail -1 $O/bench_default.log | cut -c1-400
fi
[ -n "$STOP_AFTER_BENCH" ] && exit 0
for P in ${SKIP_PROF:+none} ${SKIP_PROF:-fp32 bf16}; do
  [ "$P" = none ] && break
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$P -o run --output-format csv -- \
    python3 bench.py --precision $P --steps 20 --warmup 5 --no-cpu-baseline --no-psnr --no-dropin --no-other-precision --no-native-ref --no-ngp --no-container ${LEG_ARGS---no-llff --no-sweep} \
    > $O/prof_$P.log 2>&1 || { tail -20 $O/prof_$P.log; exit 1; }
  python3 tools/prof_summary.py $O/prof_$P/run_kernel_stats.csv 28 3 > $O/prof_${P}_summary.txt 2>&1
  python3 tools/step_timeline.py $O/prof_$P/run_kernel_trace.csv > $O/step_${P}.txt 2>&1 || true
  rm -f $O/prof_$P/run_kernel_trace.csv  # (the C5 leg's trace alone is tens of MB; gpurun returns <= 64 MiB)
  echo "prof $P: $(tail -1 $O/prof_$P.log | cut -c1-200)"
done
if [ -z "$SKIP_PROF" ]; then
# the reference's AMP loop body under autocast(float16) (fp16 build) and autocast(bfloat16) (bf16 build), kernel stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_amp -o run --output-format csv -- python3 tools/amp_kernels_ab.py \
  > $O/amp_ab.log 2>&1 || { tail -20 $O/amp_ab.log; exit 1; }
python3 tools/prof_summary.py $O/prof_amp/run_kernel_stats.csv 40 3 > $O/prof_amp_summary.txt 2>&1
rm -f $O/prof_amp/run_kernel_trace.csv
grep -E "^(fp16|bf16)" $O/amp_ab.log
fi
[ -n "$STOP_AFTER_PROF" ] && exit 0
if [ -z "$FULL_PMC_ONLY" ]; then
# the per-kernel PMC passes need only the C2 / C3 legs (the full-bench pass at the end runs every leg)
export LEG_ARGS="--no-llff --no-sweep"
PMC_OUT=$O/pmc_fp32 PMC_BENCH_ARGS="--no-dropin --no-other-precision --no-native-ref" bash tools/pmc_traffic.sh > $O/pmc_fp32.txt 2>&1 || { tail -20 $O/pmc_fp32.txt; exit 1; }
PMC_OUT=$O/pmc_bf16 PMC_PRECISION=bf16fused PMC_BENCH_ARGS="--precision bf16 --no-dropin --no-other-precision" bash tools/pmc_traffic.sh > $O/pmc_bf16.txt 2>&1 || { tail -20 $O/pmc_bf16.txt; exit 1; }
PMC_OUT=$O/pmc_mfma PMC_BENCH_ARGS="--no-other-precision --no-native-ref" bash tools/pmc_mfma_bench.sh > $O/pmc_mfma.txt 2>&1 || { tail -20 $O/pmc_mfma.txt; exit 1; }
for f in $O/pmc_fp32.txt $O/pmc_bf16.txt $O/pmc_mfma.txt; do tail -n 3 $f; done
find $O/pmc_fp32 $O/pmc_bf16 $O/pmc_mfma -name "*.csv" -size +4M -delete 2>/dev/null
VARIANTS=split bash tools/pmc_split.sh > $O/pmc_split.txt 2>&1 || { tail -20 $O/pmc_split.txt; exit 1; }
tail -n 4 $O/pmc_split.txt | cut -c1-200
find $O gpurun_out/pmc_split_split -name "*.csv" -size +4M -delete 2>/dev/null
unset LEG_ARGS
fi
[ -n "$SKIP_FULL_PMC" ] && exit 0
# one PMC pass over the whole default bench (every leg: C2, C3 + drop-ins, C4, C5 sweep, NGP, container, PSNR) with the
# counters on the first 100 dispatches of each of this library's MLP kernels (DESIGN.md §4 "rocprofv3 PMC": the kernel
# filter alone still faulted, 800 steps into the fp32 PSNR training)
F="x6|gemm|bwd_layer|mlp_fwd_fused|tail|color_bwd|head_bwd|reduce_"
timeout -s KILL 1000 rocprofv3 --kernel-include-regex "$F" --kernel-iteration-range "${PMC_ITER:-[1-100]}" --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d $O/pmc_full -o run -- python3 bench.py > $O/pmc_full_bench.log 2>&1
rc=$?; echo "PMC pass over the full bench: rc=$rc"; tail -1 $O/pmc_full_bench.log | cut -c1-300
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/r05/pmc_full/**/*counter_collection.csv", recursive=True):
    d = set(r["Dispatch_Id"] for r in csv.DictReader(open(f)))
    print("counted dispatches:", len(d))
for f in glob.glob("gpurun_out/r05/pmc_full/**/*kernel_trace.csv", recursive=True):
    print("traced dispatches:", sum(1 for _ in open(f)) - 1)
PY
rm -rf $O/pmc_full/*.csv $O/pmc_full/*/*.csv 2>/dev/null
exit $rc
