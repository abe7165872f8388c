"""One train step's kernel timeline from a rocprofv3 kernel-trace CSV: a complete step between two pick_pixels
launches (start, end, duration in us relative to the step start; queue; workgroups; kernel).

Which step: argv[2] = "mid" (default: the middle step of the trace, inside bench.py's timed region) or "last" (the
last complete step: one of bench.py's --timing-steps, whose fine-net launches are bracketed by HIP events — each
event record shows as ~5 us of idle GPU time between the launches)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
which = sys.argv[2] if len(sys.argv) > 2 else "mid"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "pick_pixels" in r["Kernel_Name"]]
k = len(idx) // 2 if which == "mid" else len(idx) - 3
a, b = idx[k], idx[k + 1]
t0 = int(rows[a]["Start_Timestamp"])
print(f"step {k} of {len(idx)} pick_pixels launches ({which})")
for r in rows[a:b]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    e = (int(r["End_Timestamp"]) - t0) / 1e3
    wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
    print(f"{s:9.1f} {e:9.1f} {e - s:8.1f} q{r['Queue_Id']} {wg:6d} {r['Kernel_Name'][:90]}")
print(f"step: {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us")
