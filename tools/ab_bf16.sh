#!/bin/bash
# A/B of the bf16 bench (C3) between the in-tree library and exp/$VARIANT.so, alternating three times on one box.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/abb && export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in base ${VARIANT:-rot}; do
    if [ $v = base ]; then L=""; else L="NERF_AMD_LIB=$PWD/exp/$v.so"; fi
    env $L timeout -k 10 200 python bench.py --precision bf16 --no-cpu-baseline --no-psnr > gpurun_out/abb/b_$v.log 2>&1 || { tail -20 gpurun_out/abb/b_$v.log; exit 1; }
    echo "$rep $v $(tail -1 gpurun_out/abb/b_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]["classes"]; print(d["value"], d["ms_per_step"], {k: v["mean_launch_ms"] for k, v in r.items()})')"
  done
done
