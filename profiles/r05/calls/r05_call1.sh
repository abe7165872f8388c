#!/bin/bash
# Round 5, first GPU call: the split-GEMM epilogue fences against HEAD's build, the parity suites that
# cover them, then a reproduction of the C5-leg SIGSEGV under rocprofv3 PMC with faulthandler on.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_c2_backward.py tests/test_gpu_split_gemm.py tests/test_gpu_parity.py \
  -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_c1.log 2>&1 || { tail -30 $O/pytest_c1.log; exit 1; }
tail -1 $O/pytest_c1.log
BENCH_EXTRA="--no-llff --no-sweep" VARIANTS="base new" ROUNDS=2 bash tools/ab_x6.sh > $O/ab_epi_fence.txt 2>&1 || { tail -20 $O/ab_epi_fence.txt; exit 1; }
cat $O/ab_epi_fence.txt
[ -n "$NO_REPRO" ] && exit 0
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d $O/segv_pmc -o run -- \
  python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-psnr --no-dropin --no-native-ref --no-other-precision --no-llff \
  --train-views 4 --sweep-scenes 2 --sweep-steps 3 --sweep-views 4 > $O/segv_pmc.log 2>&1
rc=$?
echo "segv repro rc=$rc"; tail -40 $O/segv_pmc.log
exit 0
