#!/bin/bash
# Round 5, call 34: the weight gradient's slab loop with whole register-set rounds and the partial round peeled
# (-DNERF_X6W_PEEL: no early drain of the prefetched loads at the loop top), alone and with the next slab's split held
# inside the second pair's MFMAs (-DNERF_X6W_SB) and scalar slab offsets (-DNERF_X6W_ADDR); bitwise checks, C2 A/B.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
for v in x6base peel peelsa; do
  NERF_AMD_LIB=exp/$v.so timeout -k 10 120 python tools/lib_outputs.py --precision fp32 --out $O/$v.pt > $O/lo_$v.log 2>&1 || { tail $O/lo_$v.log; exit 1; }
done
python tools/lib_outputs.py --compare $O/peel.pt $O/x6base.pt || true
python tools/lib_outputs.py --compare $O/peelsa.pt $O/x6base.pt || true; rm -f $O/*.pt
VARIANTS="x6base peel peelsa" ROUNDS=3 timeout -k 10 1000 bash tools/ab_x6.sh
