#!/bin/bash
# NGP MLP backward timing experiments (exp/*.so built by tools/build_exp.sh): mlp_bwd ms per variant
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out && export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  if [ $v = base ]; then L=""; else L="NERF_AMD_LIB=$PWD/exp/$v.so"; fi
  env $L timeout -k 10 120 python tools/bench_ngp.py --no-cpu-baseline > gpurun_out/expn_$v.log 2>&1 || { tail -20 gpurun_out/expn_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/expn_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernels_ms"])')"
done
