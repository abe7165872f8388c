"""One train step's kernel timeline from a rocprofv3 kernel-trace CSV: the last complete step between two
pick_pixels launches (start, end, duration in us relative to the step start; queue; workgroups; kernel)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "pick_pixels" in r["Kernel_Name"]]
a, b = idx[-3], idx[-2]
t0 = int(rows[a]["Start_Timestamp"])
for r in rows[a:b]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    e = (int(r["End_Timestamp"]) - t0) / 1e3
    wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
    print(f"{s:9.1f} {e:9.1f} {e - s:8.1f} q{r['Queue_Id']} {wg:6d} {r['Kernel_Name'][:90]}")
print(f"step: {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us")
