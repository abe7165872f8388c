#!/bin/bash
# Same-box A/B: the fp32 fine weight gradients on a third stream (--split-wgrad) with the round-6 schedule (coarse
# backward beside the fine backward), three alternated rounds of the C2 leg.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06/$1; mkdir -p $O
A="--steps 50 --warmup 8 --no-cpu-baseline --no-psnr --no-dropin --no-other-precision --no-native-ref --no-ngp --no-container --no-llff --no-sweep"
for r in 1 2 3; do
  for V in default split_wgrad; do
    F=""; [ $V = split_wgrad ] && F="--split-wgrad"
    timeout -k 10 120 python3 bench.py $A $F > $O/wg_${V}_$r.log 2>&1 || { tail -5 $O/wg_${V}_$r.log; exit 1; }
    echo "fp32 $V r$r $(tail -1 $O/wg_${V}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $O/wg_ab.txt
  done
done
