#!/bin/bash
# kernel trace of the container's per-step run (occupancy-update steps included): the kernels of one update step
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_upd -o run -- python3 tools/container_steps.py > gpurun_out/prof_upd.log 2>&1 || { tail -20 gpurun_out/prof_upd.log; exit 1; }
python3 - <<'PY'
import csv, glob, re
from collections import defaultdict
f = glob.glob("gpurun_out/prof_upd/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# update launches: the density evaluations with the largest grids
big = [r for r in rows if int(r["Grid_Size_X"]) >= 16_000_000 // 1]
t0 = int(big[-1]["Start_Timestamp"]) - 30_000_000 if big else 0
d = defaultdict(float); n = defaultdict(int)
for r in rows:
    if int(r["Grid_Size_X"]) * 1 >= 4_000_000 or "sort" in r["Kernel_Name"].lower() or "occ" in r["Kernel_Name"] or "cell" in r["Kernel_Name"]:
        k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", ""))[:70]
        d[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3; n[k] += 1
for k, v in sorted(d.items(), key=lambda x: -x[1])[:20]:
    print(f"{v:10.1f} us {n[k]:4d} {k}")
PY
