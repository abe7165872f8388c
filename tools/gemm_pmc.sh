#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/gpmc
rocprofv3 -L > gpurun_out/gpmc/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/gpmc/p1 -o run -- ./tools/gemm_bench 1 > gpurun_out/gpmc/p1.log 2>&1
echo rc=$?
tail -3 gpurun_out/gpmc/p1.log
