#!/bin/bash
# rocprof kernel stats of tools/bench_mlp.py (MLP passes alone at the C2 fine size)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out && export TMPDIR=/tmp
P=${PREC:-bf16}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mlp -o run --output-format csv -- python3 tools/bench_mlp.py --precision $P --iters 10 > gpurun_out/prof_mlp.log 2>&1 || { tail -20 gpurun_out/prof_mlp.log; exit 1; }
tail -1 gpurun_out/prof_mlp.log
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_mlp/run_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{float(r["AverageNs"])/1e3:9.1f} us avg x{int(r["Calls"]):5d}  {r["Name"][:100]}')
PY
