#!/bin/bash
# Round 5, call 5: the fp16 build after the element-access fix (tests + AMP drop-in rate), then the C5-leg SIGSEGV
# bisection: (1) the crashing command with --kernel-trace only (no PMC), (2) PMC over a long bf16-only engine run
# (no sweep: as many dispatches as the crashing run, no scene / trainer re-creation).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp16.py tests/test_gpu_dropin.py tests/test_gpu_bf16.py \
  -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest_c5.log 2>&1; rc=$?
grep -E "passed|failed|FAIL|Error|cosine|worst|GradScaler" $O/pytest_c5.log | cut -c1-400 | tail -20
[ $rc -gt 1 ] && exit 1
timeout -k 10 400 python bench.py --no-psnr --no-llff --no-sweep --no-ngp --no-container --no-cpu-baseline --no-native-ref --no-dropin > $O/bench_c5.log 2>&1 || { tail -30 $O/bench_c5.log; exit 1; }
tail -1 $O/bench_c5.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); b=d["bf16"]; print("C2", d["value"], "C3", b["value"], b["ms_per_step"], "AMP dropin", b["dropin"]["value"], b["dropin"]["ms_per_step"], b["dropin_vs_engine"])'
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/segv_kt -o run -- \
  python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-psnr --no-dropin --no-native-ref --no-other-precision \
  --no-ngp --no-container --train-views 4 --fp32-gemm split > $O/segv_kt.log 2>&1
rc=$?; echo "kernel-trace-only full sweep rc=$rc"; grep -v "^W20\|^E20" $O/segv_kt.log | grep -E "sweep|Fatal|SIGSEGV|File" | cut -c1-200 | tail -12
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r05/segv_kt/**/*kernel_trace.csv", recursive=True)
if f:
    n = sum(1 for _ in open(f[0])) - 1
    print("dispatches in the kernel-trace-only run:", n)
PY
rm -rf $O/segv_kt/*.csv $O/segv_kt/*/*.csv 2>/dev/null
[ $rc -ne 0 ] && exit 0
timeout -s KILL 700 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d $O/segv_pmc4 -o run -- \
  python3 bench.py --precision bf16 --steps 4000 --warmup 2 --timing-steps 1 --no-cpu-baseline --no-psnr --no-dropin --no-other-precision \
  --no-llff --no-sweep --no-ngp --no-container --train-views 4 > $O/segv_pmc4.log 2>&1
rc=$?; echo "PMC bf16-only 4000 steps rc=$rc"; grep -v "^W20\|^E20" $O/segv_pmc4.log | grep -E "value|Fatal|SIGSEGV|File|fused" | cut -c1-200 | tail -14
rm -rf $O/segv_pmc4/*.csv $O/segv_pmc4/*/*.csv 2>/dev/null
exit 0
