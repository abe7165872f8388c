#!/bin/bash
# Ring vs tiled split NT kernels: the split-GEMM GPU tests (bitwise ring == tiled, accuracy vs fp64), then the C2 bench
# with --fp32-gemm split (ring, default) and split_tiled, alternating.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_split_gemm.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_ring.log 2>&1 || { tail -30 gpurun_out/pytest_ring.log; exit 1; }
tail -3 gpurun_out/pytest_ring.log
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-split split_tiled}; do
    timeout -k 10 240 python bench.py --steps 20 --no-psnr --no-cpu-baseline --no-other-precision --no-dropin --no-native-ref --fp32-gemm $v > gpurun_out/ab_ring_$v.log 2>&1 || { tail -20 gpurun_out/ab_ring_$v.log; exit 1; }
    echo "ring-ab $v $(tail -1 gpurun_out/ab_ring_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["classes_ms"], r["class"], r["frac"], "loss", d["final_loss"])')"
  done
done
