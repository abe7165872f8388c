"""Container step anatomy from a rocprofv3 kernel-trace CSV: steps are delimited by pick_pixels launches (one per
step).  For the last complete steps: wall span, GPU busy time (union of kernel intervals), idle gaps, kernel count;
then the per-kernel totals of the last step and its ten largest idle gaps with the kernels either side of them.

  python tools/cont_timeline.py run_kernel_trace.csv [N_STEPS]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "pick_pixels" in r["Kernel_Name"]]
n_steps = int(sys.argv[2]) if len(sys.argv) > 2 else 22
spans = list(zip(idx[:-1], idx[1:]))[-n_steps - 1:-1]


def anatomy(a, b):
    t0 = int(rows[a]["Start_Timestamp"])
    t_end = int(rows[b]["Start_Timestamp"])
    busy, last_end, gaps = 0, t0, []
    for i in range(a, b):
        s, e = int(rows[i]["Start_Timestamp"]), int(rows[i]["End_Timestamp"])
        if s > last_end:
            gaps.append((s - last_end, i))
        busy += max(0, e - max(s, last_end))
        last_end = max(last_end, e)
    return (t_end - t0) / 1e3, busy / 1e3, gaps


for j, (a, b) in enumerate(spans):
    wall, busy, gaps = anatomy(a, b)
    print(f"step {len(idx) - 1 - len(spans) + j:3d}: wall {wall:8.1f} us  busy {busy:8.1f} us  idle {wall - busy:7.1f} us  kernels {b - a}")
# the anatomy below: the last step before the event-timed steps (bench_container times --steps more steps with HIP
# events after its timed region), i.e. spans[-(STEPS_EV + 1)]
ev = int(sys.argv[3]) if len(sys.argv) > 3 else 10
a, b = spans[-(ev + 1)]
per = defaultdict(lambda: [0.0, 0])
for i in range(a, b):
    d = (int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])) / 1e3
    k = rows[i]["Kernel_Name"][:80]
    per[k][0] += d
    per[k][1] += 1
print("\nlast step, per kernel (us, launches):")
for k, (t, c) in sorted(per.items(), key=lambda x: -x[1][0])[:30]:
    print(f"  {t:8.1f} {c:4d}  {k}")
_, _, gaps = anatomy(a, b)
print("\nlargest idle gaps of the last step (us: before -> after):")
for g, i in sorted(gaps, reverse=True)[:12]:
    print(f"  {g / 1e3:7.1f}  {rows[i - 1]['Kernel_Name'][:50]}  ->  {rows[i]['Kernel_Name'][:50]}")
heavy = max(spans[:-ev], key=lambda ab: anatomy(*ab)[1])
per = defaultdict(lambda: [0.0, 0])
for i in range(*heavy):
    d = (int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])) / 1e3
    per[rows[i]["Kernel_Name"][:80]][0] += d
    per[rows[i]["Kernel_Name"][:80]][1] += 1
print("\nheaviest step (the occupancy update's), per kernel (us, launches):")
for k, (t, c) in sorted(per.items(), key=lambda x: -x[1][0])[:20]:
    print(f"  {t:8.1f} {c:4d}  {k}")
walls = [anatomy(a, b) for a, b in spans[:-ev]]
print(f"\nmean over {len(walls)} steps: wall {sum(w for w, _, _ in walls) / len(walls):.1f} us, "
      f"busy {sum(x for _, x, _ in walls) / len(walls):.1f} us")
