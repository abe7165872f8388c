#!/bin/bash
# Round 5, call 35: the default build with the peeled weight-gradient loop (the A/B switches removed): bitwise against
# the measured variant exp/peel.so and the previous default exp/x6base.so, all GPU tests, then the C2 A/B.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
for v in def peel x6base; do
  NERF_AMD_LIB=exp/$v.so timeout -k 10 120 python tools/lib_outputs.py --precision fp32 --out $O/$v.pt > $O/lo_$v.log 2>&1 || { tail $O/lo_$v.log; exit 1; }
done
python tools/lib_outputs.py --compare $O/def.pt $O/peel.pt || true
python tools/lib_outputs.py --compare $O/def.pt $O/x6base.pt || true; rm -f $O/*.pt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu_all.log 2>&1; tail -1 $O/pytest_gpu_all.log
VARIANTS="x6base def peel" ROUNDS=2 timeout -k 10 900 bash tools/ab_x6.sh
