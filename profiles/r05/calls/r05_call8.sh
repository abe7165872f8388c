#!/bin/bash
# Round 5, call 8: fp16 tests after the bias-sum fix (scalar copy + v_dot2c); a short bench (C2 + C3 + drop-ins);
# the engine probe under the SQ PMC set for 8000 steps (the bf16-only bench crashed within 4000 under the same set).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp16.py tests/test_gpu_dropin.py tests/test_gpu_bf16.py \
  -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest_c8.log 2>&1; rc=$?
grep -E "passed|failed|FAIL|Error|cosine|worst|GradScaler|rgb" $O/pytest_c8.log | cut -c1-300 | tail -24
[ $rc -gt 1 ] && exit 1
timeout -k 10 400 python -u bench.py --no-psnr --no-sweep --no-llff --no-ngp --no-container > $O/bench_c8.log 2>&1 || exit 1
tail -1 $O/bench_c8.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['bf16']; print('C2', d['value'], d['ms_per_step'], 'C3', b.get('value'), b.get('ms_per_step'), 'dropin', {k: b['dropin'].get(k) for k in ('value','precision','ms_per_step') if k in b['dropin']}, 'c2 dropin', d.get('dropin',{}).get('value'))"
timeout -s KILL 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d $O/eprobe3 -o run -- python3 tools/pmc_engine_probe.py --precision bf16 --steps 8000 --every 250 > $O/eprobe3.log 2>&1
rc=$?; echo "engine probe 8000, SQ set: rc=$rc"; grep -v "^W20\|^E20" $O/eprobe3.log | grep -E "probe|Fatal|SIGSEGV|File" | tail -6
rm -rf $O/eprobe3/*.csv $O/eprobe3/*/*.csv 2>/dev/null
exit 0
