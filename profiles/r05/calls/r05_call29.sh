#!/bin/bash
# Round 5, call 29: the 256 x 256 weight gradient with three register sets (loads of slab it + 3 issued at iteration
# it, -DNERF_X6W_PF3) against the two-set default; bitwise check, then the C2 A/B.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
for v in x6base wpf3; do
  NERF_AMD_LIB=exp/$v.so timeout -k 10 120 python tools/lib_outputs.py --precision fp32 --out $O/$v.pt > $O/lo_$v.log 2>&1 || { tail $O/lo_$v.log; exit 1; }
done
python tools/lib_outputs.py --compare $O/wpf3.pt $O/x6base.pt; rm -f $O/*.pt
VARIANTS="x6base wpf3" ROUNDS=3 timeout -k 10 900 bash tools/ab_x6.sh
