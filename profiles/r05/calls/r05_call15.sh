#!/bin/bash
# Round 5, call 15: the multi-step AMP drop-in test; then the full-bench PMC pass again with counters on the first 100
# dispatches of each MLP kernel only (the kernel filter alone still faulted, at fp32 PSNR step ~800 of call B2).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py -m gpu -v -s --timeout 240 --timeout-method thread > $O/pytest_c15.log 2>&1; rc=$?
grep -E "passed|failed|FAIL|Error|step [0-9]|after 6" $O/pytest_c15.log | cut -c1-250 | tail -14
[ $rc -ne 0 ] && exit 1
FULL_PMC_ONLY=1 PMC_ITER="[1-100]" bash tools/r05_profiles.sh
