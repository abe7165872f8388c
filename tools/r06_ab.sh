#!/bin/bash
# A/B of the engine step between ab/$A.so (A may list several names) and the in-tree library (alternated), plus named
# tests first.   A=pre_pe PREC=bf16 TESTS="tests/x.py ..." tools/r06_ab.sh OUTDIR
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06/$1; mkdir -p $O; export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread > $O/pytest_ab.log 2>&1 || { tail -40 $O/pytest_ab.log; exit 1; }
  tail -1 $O/pytest_ab.log
fi
ARGS="--precision ${PREC:-bf16} --steps 30 --warmup 5 --no-cpu-baseline --no-psnr --no-dropin --no-other-precision --no-native-ref --no-ngp --no-container --no-llff --no-sweep"
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in $A new; do
    if [ $v = new ]; then L=""; else L="NERF_AMD_LIB=ab/$v.so"; fi
    env $L timeout -k 10 200 python bench.py $ARGS > $O/ab_${v}_$r.json 2> $O/ab_${v}_$r.err || { tail -20 $O/ab_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/ab_${v}_$r.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', d['value'], d['ms_per_step'], r.get('class'), r.get('mean_launch_ms'), {k: v.get('mean_launch_ms') for k, v in r.get('classes', {}).items()})"
  done
done
