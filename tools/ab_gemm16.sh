#!/bin/bash
# 16x16x4 fp32 trunk GEMMs (in-tree library) vs the 32x32x2 ones (exp/gemm32.so, -DNERF_GEMM32): kernel sweep,
# fp32 MLP parity tests on the new library, then bench.py alternating twice on the same box.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab16 && export TMPDIR=/tmp
O=gpurun_out/ab16
# (kernel sweep: ./tools/gemm_bench16 9)

timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_edges.py > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for rep in 1 2; do
  for v in base gemm32; do
    if [ $v = base ]; then L=""; else L="NERF_AMD_LIB=$PWD/exp/$v.so"; fi
    env $L timeout -k 10 200 python bench.py --no-cpu-baseline --no-dropin --no-psnr > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
    echo "$rep $v $(tail -1 $O/bench_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["class"], r["frac"], r["classes_ms"])')"
  done
done
