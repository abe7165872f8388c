#!/bin/bash
# Round 5, call 3: split-GEMM A/B (HEAD r04 / epilogue drain / pair barriers fwd / + input gradient / trunk.0 4-wave /
# coarse splits of 2048 rows), bench.py's own world-2 dp path, the default bench line with the new ngp / container
# legs, then the C5-leg SIGSEGV repro under rocprofv3 PMC with the C4 leg before it.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
BENCH_EXTRA="--no-llff --no-sweep" VARIANTS="base new pb pb3 k64nw4 sr2048" ROUNDS=2 bash tools/ab_x6.sh > $O/ab_c3.txt 2>&1 || { tail -20 $O/ab_c3.txt; exit 1; }
cat $O/ab_c3.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py -m gpu -v -s --timeout 300 --timeout-method thread -k bench > $O/pytest_dp_bench.log 2>&1; rc=$?
grep -E "passed|failed|PASS|FAIL|Error|world_size" $O/pytest_dp_bench.log | cut -c1-600 | tail -8
[ $rc -gt 1 ] && exit 1
timeout -k 10 560 python bench.py --no-psnr > $O/bench_nopsnr.log 2>&1 || { tail -30 $O/bench_nopsnr.log; exit 1; }
tail -1 $O/bench_nopsnr.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["classes_ms"]); print("bf16", d["bf16"]["value"], "dropin", d["bf16"].get("dropin",{}).get("value")); print("ngp", {k: d["ngp"][k] for k in ("value","ms_per_step","kernels_ms","atomic_roofline")}); print("container", {k: d["container"][k] for k in ("value","ms_per_step","roofline","dominant")}); print("cpu", d["ngp"]["cpu_baseline"], d["container"]["cpu_baseline"])'
[ -n "$NO_REPRO" ] && exit 0
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d $O/segv_pmc2 -o run -- \
  python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-psnr --no-dropin --no-native-ref --no-other-precision \
  --no-ngp --no-container --train-views 4 --sweep-scenes 2 --sweep-steps 3 > $O/segv_pmc2.log 2>&1
rc=$?
echo "segv repro2 rc=$rc"; grep -v "^W20\|^E20" $O/segv_pmc2.log | cut -c1-300 | tail -40
exit 0
