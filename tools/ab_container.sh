#!/bin/bash
# A/B of container + NGP benches between the in-tree library and exp/$VARIANT.so (same box), alternating twice
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2; do
  for v in base ${VARIANT:-oldhash}; do
    if [ $v = base ]; then L=""; else L="NERF_AMD_LIB=$PWD/exp/$v.so"; fi
    env $L timeout -k 10 200 python tools/bench_ngp.py --no-cpu-baseline > gpurun_out/ab_ngp_$v.log 2>&1 || { tail -20 gpurun_out/ab_ngp_$v.log; exit 1; }
    env $L timeout -k 10 300 python tools/bench_container.py --no-cpu-baseline --steps 48 > gpurun_out/ab_c_$v.log 2>&1 || { tail -20 gpurun_out/ab_c_$v.log; exit 1; }
    echo "$rep $v ngp $(tail -1 gpurun_out/ab_ngp_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernels_ms"])') container $(tail -1 gpurun_out/ab_c_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
