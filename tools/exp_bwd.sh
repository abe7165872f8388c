#!/bin/bash
# bf16 layer-backward ablations (exp/*.so built by tools/build_exp.sh with -DNERF_EXP_BWD_*): per variant the MLP
# backward time (tools/bench_mlp.py) and the rocprof average of the fused layer kernel.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/expb && export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  if [ $v = base ]; then L=""; else L="NERF_AMD_LIB=$PWD/exp/$v.so"; fi
  env $L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/expb/$v -o run --output-format csv -- \
    python3 tools/bench_mlp.py --precision bf16 --iters 10 > gpurun_out/expb/$v.log 2>&1 || { tail -20 gpurun_out/expb/$v.log; exit 1; }
  k=$(python3 - "$v" <<'PY'
import csv, glob, sys
v = sys.argv[1]
out = []
for f in glob.glob(f"gpurun_out/expb/{v}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if any(k in n for k in ("bwd_layer", "fwd_fused", "bwd_tail", "wgrad_bf16", "reduce_fused")):
            out.append(f"{n.split('(')[0].split('::')[-1][:28]}={float(r['AverageNs'])/1e3:.1f}us")
print(" ".join(sorted(out)))
PY
)
  echo "$v $(tail -1 gpurun_out/expb/$v.log | cut -c1-160) | $k"
done
