#!/bin/bash
# Round-6 GPU check: named tests first (fast feedback), then every -m gpu test, smoke(), the default bench line.
# Usage: tools/r06_check.sh OUTDIR ["pytest node ids for the first pass"]  (NO_BENCH=1 skips the bench)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/$1; mkdir -p $O; export TMPDIR=/tmp
if [ -n "$2" ]; then
  timeout -k 10 400 python -u -m pytest $2 -x -v --timeout 300 --timeout-method thread > $O/pytest_first.log 2>&1 || { tail -40 $O/pytest_first.log; exit 1; }
  tail -1 $O/pytest_first.log
fi
[ -n "$NO_ALL" ] || { timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_all.log 2>&1 || { tail -30 $O/pytest_gpu_all.log; exit 1; }; tail -1 $O/pytest_gpu_all.log; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default_stderr.txt || { tail -30 $O/bench_default_stderr.txt; exit 1; }
cut -c1-400 $O/bench_default.json
