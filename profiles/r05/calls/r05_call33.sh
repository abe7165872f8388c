#!/bin/bash
# Round 5, call 33: the narrow weight gradient (trunk.0, trunk.4 encoding columns) with raw-register bias sums (a different order for trunk.0's bias)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
for v in x6base nbraw; do
  NERF_AMD_LIB=exp/$v.so timeout -k 10 120 python tools/lib_outputs.py --precision fp32 --out $O/$v.pt > $O/lo_$v.log 2>&1 || { tail $O/lo_$v.log; exit 1; }
done
python tools/lib_outputs.py --compare $O/nbraw.pt $O/x6base.pt || true; rm -f $O/*.pt
VARIANTS="x6base nbraw" ROUNDS=3 timeout -k 10 900 bash tools/ab_x6.sh
NERF_AMD_LIB=exp/nbraw.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_nbraw.log 2>&1; tail -1 $O/pytest_nbraw.log
