#!/bin/bash
# Round 5, call 30: the 256 x 256 weight gradient with the bias-column sums shared by both wave halves
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
for v in x6base wbias; do
  NERF_AMD_LIB=exp/$v.so timeout -k 10 120 python tools/lib_outputs.py --precision fp32 --out $O/$v.pt > $O/lo_$v.log 2>&1 || { tail $O/lo_$v.log; exit 1; }
done
python tools/lib_outputs.py --compare $O/wbias.pt $O/x6base.pt; rm -f $O/*.pt
VARIANTS="x6base wbias" ROUNDS=3 timeout -k 10 900 bash tools/ab_x6.sh
