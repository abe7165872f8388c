#!/bin/bash
# A/B of split-GEMM experiment builds (tools/build_exp.sh NAME FLAGS -> exp/NAME.so) on the C2 bench, alternating
# variants so that clock drift hits all of them.  Usage: VARIANTS="x6base x6even" ROUNDS=2 tools/ab_x6.sh
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out && export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-x6base}; do
    NERF_AMD_LIB=exp/$v.so timeout -k 10 240 python bench.py --steps 20 --no-psnr --no-cpu-baseline --no-other-precision --no-dropin ${BENCH_EXTRA:-} > gpurun_out/ab_$v.log 2>&1 || { tail -20 gpurun_out/ab_$v.log; exit 1; }
    echo "x6-ab $v $(tail -1 gpurun_out/ab_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["classes_ms"], r["class"], r["frac"], "loss", d["final_loss"])')"
  done
done
