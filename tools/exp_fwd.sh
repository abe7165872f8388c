#!/bin/bash
# fused bf16 forward timing experiments (exp/*.so from tools/build_exp.sh): fwd_infer / fwd_train / bwd ms per variant
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out && export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  if [ $v = base ]; then L=""; else L="NERF_AMD_LIB=$PWD/exp/$v.so"; fi
  env $L timeout -k 10 120 python tools/bench_mlp.py --precision bf16 > gpurun_out/expf_$v.log 2>&1 || { tail -20 gpurun_out/expf_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/expf_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d.get("fwd_infer_ms"), d.get("fwd_train_ms"), d.get("bwd_ms"))')"
done
