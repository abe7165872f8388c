#!/bin/bash
# Round 5, call 16: where the production container step's time goes — rocprof kernel stats + trace of
# tools/bench_container.py (48 timed steps after 40 warm-up), and the step timeline of the last steps.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_cont -o run --output-format csv -- \
  python3 tools/bench_container.py --steps 48 --warmup 40 --no-cpu-baseline > $O/prof_cont.log 2>&1 || { tail -20 $O/prof_cont.log; exit 1; }
tail -1 $O/prof_cont.log | cut -c1-300
python3 tools/prof_summary.py $O/prof_cont/run_kernel_stats.csv 40 48 > $O/prof_cont_summary.txt 2>&1
head -45 $O/prof_cont_summary.txt | cut -c1-200
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r05/prof_cont/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last 5 steps: from the 5th-last FlatAdam-like launch; print busy vs span
t = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]) for r in rows]
span0, span1 = t[-1][1] - 25_000_000, t[-1][1]
sel = [x for x in t if x[0] >= span0]
busy, cur_s, cur_e = 0, None, None
for s, e, _ in sel:
    if cur_e is None or s > cur_e:
        if cur_e is not None: busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print(f"last 25 ms of the trace: {len(sel)} dispatches, GPU busy {busy/1e6:.2f} ms of {(span1-span0)/1e6:.2f} ms")
gaps = []
for a, b in zip(sel, sel[1:]):
    if b[0] > a[1]: gaps.append((b[0] - a[1], a[2], b[2]))
gaps.sort(reverse=True)
for g in gaps[:12]: print(f"gap {g[0]/1e3:8.1f} us after {g[1]} -> {g[2]}")
PY
rm -f $O/prof_cont/run_kernel_trace.csv
