#!/bin/bash
# Round 5, call 4: fp16-build spill fixes (tests + the AMP drop-in rate), the production-form exchange events at world 2,
# then the round-4 crashing PMC command verbatim (full default C5 sweep: 8 scenes x 500 steps) with faulthandler on.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp16.py tests/test_gpu_dropin.py tests/test_gpu_bf16.py tests/test_gpu_dp.py \
  -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest_c4.log 2>&1; rc=$?
grep -E "passed|failed|FAIL|Error|cosine|worst|GradScaler|world_size" $O/pytest_c4.log | cut -c1-700 | tail -30
[ $rc -gt 1 ] && exit 1
timeout -k 10 400 python bench.py --no-psnr --no-llff --no-sweep --no-ngp --no-container --no-cpu-baseline --no-native-ref > $O/bench_c4.log 2>&1 || { tail -30 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("C2", d["value"], d["ms_per_step"], d["roofline"]["classes_ms"], "dropin", d["dropin"]["value"]); b=d["bf16"]; print("C3", b["value"], b["ms_per_step"], "AMP dropin", b["dropin"]["value"], b["dropin"]["ms_per_step"], b["dropin_vs_engine"])'
[ -n "$NO_REPRO" ] && exit 0
timeout -s KILL 700 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d $O/segv_pmc3 -o run -- \
  python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-psnr --no-dropin --no-native-ref --no-other-precision \
  --no-ngp --no-container --train-views 4 --fp32-gemm split > $O/segv_pmc3.log 2>&1
rc=$?
echo "segv repro3 rc=$rc"; grep -v "^W20\|^E20" $O/segv_pmc3.log | cut -c1-300 | tail -60
rm -rf $O/segv_pmc3/*.csv
exit 0
