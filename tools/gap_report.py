"""GPU idle gaps in a rocprofv3 kernel-trace CSV: busy fraction (union of kernel intervals over the span) of a
window and the largest gaps with the kernels on either side — where the host (syncs, Python launch cost) is
the bottleneck.  Usage: python tools/gap_report.py run_kernel_trace.csv [start_frac 0.6] [end_frac 0.95] [top 25]"""
import csv
import sys
from collections import Counter


def main():
    path = sys.argv[1]
    f0 = float(sys.argv[2]) if len(sys.argv) > 2 else 0.6
    f1 = float(sys.argv[3]) if len(sys.argv) > 3 else 0.95
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 25
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[int(len(rows) * f0):int(len(rows) * f1)]
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]) for r in rows]
    span = iv[-1][1] - iv[0][0]
    busy, cur_s, cur_e, gaps, prev = 0, iv[0][0], iv[0][1], [], iv[0][2]
    for s, e, n in iv[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, prev, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev = n if e >= cur_e else prev
    busy += cur_e - cur_s
    print(f"{len(iv)} kernels over {span / 1e6:.2f} ms: busy {busy / 1e6:.2f} ms ({busy / span:.1%}), "
          f"idle {(span - busy) / 1e6:.2f} ms in {len(gaps)} gaps")
    per = Counter()
    for g, a, b in gaps:
        per[(a, b)] += g
    print("idle time by (kernel before -> kernel after), top:")
    for (a, b), g in per.most_common(top):
        print(f"  {g / 1e6:8.3f} ms  {a}  ->  {b}")


if __name__ == "__main__":
    main()
