#!/bin/bash
# MFMA utilisation of the bench's own kernels (fp32 C2 step): SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES and
# GRBM_GUI_ACTIVE in one PMC pass (kernel trace only, no other tracing), parsed per kernel by tools/gemm_pmc_parse.py.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc_mfma}
mkdir -p $OUT
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d $OUT/p1 -o run -- \
  python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-psnr --no-dropin --no-ngp --no-container ${LEG_ARGS:---sweep-steps 50} --train-views 4 $PMC_BENCH_ARGS > $OUT/p1.log 2>&1 || { tail -20 $OUT/p1.log; exit 1; }
python3 tools/gemm_pmc_parse.py $OUT/p1 | grep -v rocclr > $OUT/summary.txt
cat $OUT/summary.txt | cut -c1-200
