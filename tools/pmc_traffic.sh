#!/bin/bash
# HBM traffic of the bench's kernels from rocprofv3 PMC counters: FETCH_SIZE and WRITE_SIZE in separate
# passes (MI355X_MICROARCH.md: TCC slots — they do not fit one pass), kernel-trace only, no other tracing.
set -o pipefail
# Counters are collected on this library's MLP kernels only (PMC_FILTER -> --kernel-include-regex; PMC_FILTER= collects
# on every dispatch): with every dispatch counted, rocprofv3 7.2 faults inside librocprofiler-sdk after a few hundred to
# a few thousand train steps (DESIGN.md §4 "rocprofv3 PMC"), so round 4 had to drop the C4 / C5 legs.  The filter
# lowers the rate; these short passes (2-3 steps per leg) stay far below it.  A pass over the whole bench also needs
# --kernel-iteration-range (tools/r05_profiles.sh).  LEG_ARGS adds leg flags (e.g. "--no-llff --no-sweep").
PMC_FILTER=${PMC_FILTER-"x6|gemm|bwd_layer|mlp_fwd_fused|tail|color_bwd|head_bwd|reduce_"}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc}
mkdir -p $OUT
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 ${PMC_FILTER:+--kernel-include-regex "$PMC_FILTER"} --pmc $C --kernel-trace --output-format csv -d $OUT/$C -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-psnr --no-ngp --no-container $LEG_ARGS --train-views 4 $PMC_BENCH_ARGS > $OUT/$C.log 2>&1 || { tail -20 $OUT/$C.log; exit 1; }
done
python3 tools/pmc_parse.py $OUT $PMC_PRECISION
