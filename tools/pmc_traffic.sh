#!/bin/bash
# (C4 / C5 legs run again, round 5: the rocprofv3 PMC SIGSEGV of round 4 is traced in DESIGN.md §4; LEG_ARGS bounds the
# sweep, "--no-llff --no-sweep" skips both)
# HBM traffic of the bench's kernels from rocprofv3 PMC counters: FETCH_SIZE and WRITE_SIZE in separate
# passes (MI355X_MICROARCH.md: TCC slots — they do not fit one pass), kernel-trace only, no other tracing.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc}
mkdir -p $OUT
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/$C -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-psnr --no-ngp --no-container ${LEG_ARGS:---sweep-steps 50} --train-views 4 $PMC_BENCH_ARGS > $OUT/$C.log 2>&1 || { tail -20 $OUT/$C.log; exit 1; }
done
python3 tools/pmc_parse.py $OUT $PMC_PRECISION
