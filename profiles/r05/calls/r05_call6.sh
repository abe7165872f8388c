#!/bin/bash
# Round 5, call 6: fp16 tests after the dot2 selector fix; then the dispatch-count probe under rocprofv3 PMC with no
# code of this repository loaded (tools/pmc_dispatch_probe.py).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp16.py tests/test_gpu_dropin.py \
  -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest_c6.log 2>&1; rc=$?
grep -E "passed|failed|FAIL|Error|cosine|worst|GradScaler|rgb" $O/pytest_c6.log | cut -c1-300 | tail -24
[ $rc -gt 1 ] && exit 1
timeout -k 10 400 python bench.py --no-psnr --no-llff --no-sweep --no-ngp --no-container --no-cpu-baseline --no-native-ref --no-dropin > $O/bench_c6.log 2>&1 || { tail -30 $O/bench_c6.log; exit 1; }
tail -1 $O/bench_c6.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); b=d["bf16"]; print("C2", d["value"], "C3", b["value"], b["ms_per_step"], "AMP dropin", b["dropin"]["value"], b["dropin"]["ms_per_step"], b["dropin_vs_engine"])'
timeout -s KILL 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d $O/probe_pmc -o run -- python3 tools/pmc_dispatch_probe.py --n 200000 --every 2000 > $O/probe_pmc.log 2>&1
rc=$?; echo "probe rc=$rc"; grep -v "^W20\|^E20" $O/probe_pmc.log | grep -E "probe|Fatal|SIGSEGV" | tail -6
rm -rf $O/probe_pmc/*.csv $O/probe_pmc/*/*.csv 2>/dev/null
exit 0
