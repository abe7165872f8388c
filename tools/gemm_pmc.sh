#!/bin/bash
# SQ/GRBM counters of the GEMM micro-benchmark variants (one counter pass, kernel trace only).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
BIN=${1:-./tools/gemm_bench2}
mkdir -p gpurun_out/gpmc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/gpmc/p1 -o run -- $BIN 1 > gpurun_out/gpmc/p1.log 2>&1
echo rc=$?
tail -12 gpurun_out/gpmc/p1.log
python3 tools/gemm_pmc_parse.py gpurun_out/gpmc/p1
