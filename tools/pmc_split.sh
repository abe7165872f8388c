#!/bin/bash
# Where the split NT GEMMs' wave cycles go: one PMC pass per fp32 engine (--fp32-gemm: split = default, native_dgrad, native) over a short C2
# bench: parked (SQ_WAIT_ANY: s_waitcnt / barrier), issue-stalled (SQ_WAIT_INST_ANY, LDS part SQ_WAIT_INST_LDS),
# issuing (SQ_ACTIVE_INST_ANY), MFMA busy and clock per kernel (tools/gemm_pmc_parse.py).
set -o pipefail
# Counters are collected on this library's MLP kernels only (PMC_FILTER -> --kernel-include-regex; PMC_FILTER= collects
# on every dispatch): with every dispatch counted, rocprofv3 7.2 faults inside librocprofiler-sdk after a few hundred to
# a few thousand train steps (DESIGN.md §4 "rocprofv3 PMC"), so round 4 had to drop the C4 / C5 legs.  The filter
# lowers the rate; these short passes (2-3 steps per leg) stay far below it.  A pass over the whole bench also needs
# --kernel-iteration-range (tools/r05_profiles.sh).  LEG_ARGS adds leg flags (e.g. "--no-llff --no-sweep").
PMC_FILTER=${PMC_FILTER-"x6|gemm|bwd_layer|mlp_fwd_fused|tail|color_bwd|head_bwd|reduce_"}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for v in ${VARIANTS:-split}; do
  OUT=gpurun_out/pmc_split_$v
  mkdir -p $OUT
  timeout -s KILL 240 rocprofv3 ${PMC_FILTER:+--kernel-include-regex "$PMC_FILTER"} --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d $OUT/p1 -o run -- \
    python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-psnr --no-dropin --no-native-ref --no-other-precision --no-ngp --no-container $LEG_ARGS --train-views 4 --fp32-gemm $v > $OUT/p1.log 2>&1 || { tail -20 $OUT/p1.log; exit 1; }
  python3 tools/gemm_pmc_parse.py $OUT/p1 | grep -v rocclr | grep -E "x6|wgrad" > $OUT/summary.txt
  echo "== $v"; cut -c1-330 $OUT/summary.txt
done
