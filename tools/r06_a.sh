#!/bin/bash
# Round-6 check: named tests first, every -m gpu test, smoke, the container step eager vs graph (alternated), the
# default bench line.  Usage: tools/r06_a.sh OUTDIR ["first tests"]  (NO_ALL=1 / NO_BENCH=1 / NO_CONT=1 skip legs)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06/$1; mkdir -p $O; export TMPDIR=/tmp
if [ -n "$2" ]; then
  timeout -k 10 400 python -u -m pytest $2 -x -v --timeout 300 --timeout-method thread > $O/pytest_first.log 2>&1 || { tail -40 $O/pytest_first.log; exit 1; }
  tail -1 $O/pytest_first.log
fi
[ -n "$NO_ALL" ] || { timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_all.log 2>&1 || { tail -30 $O/pytest_gpu_all.log; exit 1; }; tail -1 $O/pytest_gpu_all.log; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
if [ -z "$NO_CONT" ]; then
for mode in eager graph eager graph; do
  F="--no-graph"; [ $mode = graph ] && F="--graph"
  timeout -k 10 300 python tools/bench_container.py --no-cpu-baseline --steps 48 --warmup 40 $F > $O/bc_$mode.log 2>&1 || { tail -30 $O/bc_$mode.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bc_$mode.log').read().strip().splitlines()[-1]); print('$mode', d['value'], d['ms_per_step'], d['host_ms_per_step'], d['kernels_ms_per_step'], d['samples_per_step'], d.get('graph'))"
done
fi
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default_stderr.txt || { tail -30 $O/bench_default_stderr.txt; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); print('C2', d['value'], d['ms_per_step'], 'C3', d['bf16']['value'], 'cont', d['container']['value'], 'ngp', d['ngp']['value'], 'roof', d['roofline']['frac'])"
