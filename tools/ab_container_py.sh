#!/bin/bash
# A/B of tools/bench_container.py between the in-tree Python package and an older package copy in exp/old (same .so)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/abc && export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in base old; do
    if [ $v = base ]; then B=tools/bench_container.py; else B=exp/old/tools/bench_container.py; fi
    timeout -k 10 250 python $B --no-cpu-baseline > gpurun_out/abc/b_$v.log 2>&1 || { tail -20 gpurun_out/abc/b_$v.log; exit 1; }
    echo "$rep $v $(tail -1 gpurun_out/abc/b_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
