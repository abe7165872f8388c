#!/bin/bash
# PMC passes (one counter group per run) over tools/bench_mlp.py: HBM bytes and L2 hit rate per MLP kernel launch
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmc_mlp
mkdir -p $OUT
P=${PREC:-bf16}
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" ${EXTRA_PMC}; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
    python3 tools/bench_mlp.py --precision $P --iters 2 > $OUT/p$i.log 2>&1 || { tail -20 $OUT/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
out = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc_mlp/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r.get("Kernel_Name", "")[:60]
        out[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, d in out.items():
    if not any(k in n for k in ("bwd_layer", "fused", "wgrad", "gemm_nt")):
        continue
    s = "  ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(d.items()))
    print(f"{n:60s} {s}")
PY
