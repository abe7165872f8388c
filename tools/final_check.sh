#!/bin/bash
# End-of-round check at HEAD on one GPU box: every -m gpu test, smoke(), and the default bench line (gpurun_out/final).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/final; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_all.log 2>&1 || { tail -30 $O/pytest_gpu_all.log; exit 1; }
tail -1 $O/pytest_gpu_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 560 python bench.py > $O/bench_default.log 2>&1 || { tail -30 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-300
