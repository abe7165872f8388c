"""Print one train step's kernel sequence from a rocprofv3 kernel-trace CSV (start offset, duration,
queue, grid, name) — used to see which launches overlap and which are slow.
Usage: python tools/trace_step.py run_kernel_trace.csv [first_row] [count]"""
import csv
import sys


def main():
    path = sys.argv[1]
    first = int(sys.argv[2]) if len(sys.argv) > 2 else None
    count = int(sys.argv[3]) if len(sys.argv) > 3 else 80
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    t0 = int(rows[0]["Start_Timestamp"])
    if first is None:
        first = len(rows) // 2
    print(f"{len(rows)} dispatches")
    for r in rows[first:first + count]:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        e = (int(r["End_Timestamp"]) - t0) / 1e3
        print(f"{s:12.1f} {e - s:8.1f} q{r.get('Queue_Id', '')} g{r.get('Grid_Size', '')} "
              f"{r['Kernel_Name'][:70]}")


if __name__ == "__main__":
    main()
