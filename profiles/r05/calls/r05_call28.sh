#!/bin/bash
# Round 5, call 28: two knobs re-tuned on the 256 x 256 forward: activation loads after the slab's MFMAs
# (-DNERF_X6W_LATE_A) and the dot-form split residuals (-DNERF_X6_DOT2_FWD=1); bitwise checks, then the C2 A/B.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
for v in x6base latea dot2fwd; do
  NERF_AMD_LIB=exp/$v.so timeout -k 10 120 python tools/lib_outputs.py --precision fp32 --out $O/$v.pt > $O/lo_$v.log 2>&1 || { tail $O/lo_$v.log; exit 1; }
done
python tools/lib_outputs.py --compare $O/latea.pt $O/x6base.pt; python tools/lib_outputs.py --compare $O/dot2fwd.pt $O/x6base.pt; rm -f $O/*.pt
VARIANTS="x6base latea dot2fwd" ROUNDS=2 timeout -k 10 900 bash tools/ab_x6.sh
