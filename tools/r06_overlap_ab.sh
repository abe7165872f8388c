#!/bin/bash
# Same-box A/B of the two-stream schedule: the coarse backward beside the fine forward (default), beside the fine
# backward, or on the main stream (--no-overlap); C3 (bf16) and C2 (fp32) legs alternated, 3 rounds.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06/$1; mkdir -p $O
A="--steps 50 --warmup 8 --no-cpu-baseline --no-psnr --no-dropin --no-other-precision --no-native-ref --no-ngp --no-container --no-llff --no-sweep"
for r in 1 2 3; do
  for P in bf16 fp32; do
    for V in fwd bwd none; do
      F="--overlap-with $V"; [ $V = none ] && F="--no-overlap"
      timeout -k 10 120 python3 bench.py --precision $P $A $F > $O/ov_${P}_${V}_$r.log 2>&1 || { tail -5 $O/ov_${P}_${V}_$r.log; exit 1; }
      echo "$P $V r$r $(tail -1 $O/ov_${P}_${V}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $O/overlap_ab.txt
    done
  done
done
