#!/bin/bash
# SQ counters of the fused bf16 backward layer kernel (tools/bench_mlp.py), one counter group per run
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmc_bwd
mkdir -p $OUT
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  for v in ${VARIANTS:-base}; do
    if [ $v = base ]; then L=""; else L="NERF_AMD_LIB=$PWD/exp/$v.so"; fi
    env $L timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/${v}_p$i -o run -- \
      python3 tools/bench_mlp.py --precision bf16 --iters 2 > $OUT/${v}_p$i.log 2>&1 || { tail -20 $OUT/${v}_p$i.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, collections, os
for d in sorted(glob.glob("gpurun_out/pmc_bwd/*_p*")):
    if not os.path.isdir(d): continue
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r.get("Kernel_Name", "")
            if "bwd_layer" in n or "bwd_tail" in n or "fwd_fused" in n:
                out[n[:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for n, dd in out.items():
        print(os.path.basename(d), n, "  ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(dd.items())))
PY
