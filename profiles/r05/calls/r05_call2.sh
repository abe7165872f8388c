#!/bin/bash
# Round 5, second GPU call: fp16 build of the fused MLP (AMP drop-in) tests, bf16 regression, split-GEMM epilogue A/B,
# and the C5-leg SIGSEGV repro with the C4 leg before it (as in the crashing run).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_fp16.py tests/test_gpu_dropin.py tests/test_gpu_bf16.py tests/test_gpu_c2_backward.py \
  -m gpu -v -s --timeout 200 --timeout-method thread > $O/pytest_c2.log 2>&1; rc=$?
grep -E "passed|failed|PASS|FAIL|Error|cosine|relative|rgb|GradScaler" $O/pytest_c2.log | tail -60
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit 1
BENCH_EXTRA="--no-llff --no-sweep" VARIANTS="base new pb pb3 k64nw4 sr2048" ROUNDS=2 bash tools/ab_x6.sh > $O/ab_epi_fence2.txt 2>&1 || { tail -20 $O/ab_epi_fence2.txt; exit 1; }
cat $O/ab_epi_fence2.txt
[ -n "$NO_REPRO" ] && exit 0
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d $O/segv_pmc2 -o run -- \
  python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-psnr --no-dropin --no-native-ref --no-other-precision \
  --train-views 4 --sweep-scenes 2 --sweep-steps 3 > $O/segv_pmc2.log 2>&1
rc=$?
echo "segv repro2 rc=$rc"; grep -v "^W20\|^E20" $O/segv_pmc2.log | cut -c1-300 | tail -40
exit 0
