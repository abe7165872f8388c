#!/bin/bash
# Round 5, call 31: the weight gradient's bias columns summed from the raw fp32 staging registers (-DNERF_X6W_BIAS_RAW; a different summation order)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
for v in x6base wbraw; do
  NERF_AMD_LIB=exp/$v.so timeout -k 10 120 python tools/lib_outputs.py --precision fp32 --out $O/$v.pt > $O/lo_$v.log 2>&1 || { tail $O/lo_$v.log; exit 1; }
done
python tools/lib_outputs.py --compare $O/wbraw.pt $O/x6base.pt || true; rm -f $O/*.pt
VARIANTS="x6base wbraw" ROUNDS=3 timeout -k 10 900 bash tools/ab_x6.sh
NERF_AMD_LIB=exp/wbraw.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_wbraw.log 2>&1; tail -1 $O/pytest_wbraw.log
