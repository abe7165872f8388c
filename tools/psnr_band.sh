#!/bin/bash
# PSNR noise band of the C2 fp32 trajectory: tools/train_psnr.py to 3000 steps, 8 held-out
# 800x800 views, same seed-0 weights and batches, jitter seeds 0..N-1; each library variant in VARIANTS
# (exp/<name>.so, "default" = lib/libnerf_amd.so).  Output: gpurun_out/psnr_band/<variant>_s<seed>.jsonl
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/psnr_band; mkdir -p $O
for s in $(seq 0 $((${SEEDS:-3} - 1))); do
  for v in ${VARIANTS:-default}; do
    L=""; [ "$v" != default ] && L="exp/$v.so"
    NERF_AMD_LIB=${L:-nerf-sys_amd/lib/libnerf_amd.so} timeout -k 10 240 python tools/train_psnr.py --steps 3000 --eval-every 3000 \
      --test-views 8 --jitter-seed $s --out $O/${v}_s$s.jsonl > $O/${v}_s$s.log 2>&1 || { tail -20 $O/${v}_s$s.log; exit 1; }
    echo "psnr-band $v seed $s $(tail -1 $O/${v}_s$s.jsonl)"
  done
done
