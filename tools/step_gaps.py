"""Per-step GPU idle analysis from a rocprofv3 kernel-trace CSV: steps are delimited by a marker kernel (the
optimizer's, default adam_kernel); prints busy / idle per step and the idle gaps of the median step with the
kernels around them.  Usage: python tools/step_gaps.py run_kernel_trace.csv [marker] [min_gap_us]"""
import csv
import statistics
import sys


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "adam_kernel"
    min_gap = float(sys.argv[3]) if len(sys.argv) > 3 else 15.0
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    marks = [i for i, (_, _, n) in enumerate(iv) if marker in n]
    steps = []
    for a, b in zip(marks[:-1], marks[1:]):
        seg = iv[a + 1:b + 1]
        span = seg[-1][1] - iv[a][1]
        cur, gaps, busy = iv[a][1], [], 0
        prev = iv[a][2]
        for s, e, n in seg:
            if s > cur:
                gaps.append(((s - cur) / 1e3, prev, n))
            busy += max(0, e - max(s, cur))
            if e > cur:
                cur, prev = e, n
        steps.append((span / 1e6, busy / 1e6, gaps, len(seg)))
    spans = [s[0] for s in steps]
    print(f"{len(steps)} steps; span ms: median {statistics.median(spans):.3f} min {min(spans):.3f}")
    med = sorted(steps, key=lambda s: s[0])[len(steps) // 2]
    print(f"median step: {med[0]:.3f} ms, busy {med[1]:.3f} ms, {med[3]} kernels, "
          f"idle {med[0] - med[1]:.3f} ms in {len(med[2])} gaps")
    for g, a, b in med[2]:
        if g >= min_gap:
            print(f"  {g:8.1f} us  {a[:55]}  ->  {b[:55]}")


if __name__ == "__main__":
    main()
