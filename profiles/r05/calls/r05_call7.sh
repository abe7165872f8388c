#!/bin/bash
# Round 5, call 7: fp16 tests after the bias-sum rewrite; the PMC failure bisection with the engine probe (progress
# every 100 steps): (1) one GRBM counter, (2) the 9-counter SQ set of tools/pmc_split.sh.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp16.py tests/test_gpu_dropin.py tests/test_gpu_bf16.py \
  -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest_c7.log 2>&1; rc=$?
grep -E "passed|failed|FAIL|Error|cosine|worst|GradScaler|rgb" $O/pytest_c7.log | cut -c1-300 | tail -24
[ $rc -gt 1 ] && exit 1
timeout -s KILL 400 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/eprobe1 -o run -- \
  python3 tools/pmc_engine_probe.py --precision bf16 --steps 3000 --every 100 > $O/eprobe1.log 2>&1
rc=$?; echo "engine probe, GRBM only: rc=$rc"; grep -v "^W20\|^E20" $O/eprobe1.log | grep -E "probe|Fatal|SIGSEGV|File" | tail -5
rm -rf $O/eprobe1/*.csv $O/eprobe1/*/*.csv 2>/dev/null
[ $rc -ne 0 ] && exit 0
timeout -s KILL 500 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d $O/eprobe2 -o run -- python3 tools/pmc_engine_probe.py --precision bf16 --steps 3000 --every 100 > $O/eprobe2.log 2>&1
rc=$?; echo "engine probe, SQ set: rc=$rc"; grep -v "^W20\|^E20" $O/eprobe2.log | grep -E "probe|Fatal|SIGSEGV|File" | tail -6
rm -rf $O/eprobe2/*.csv $O/eprobe2/*/*.csv 2>/dev/null
exit 0
