"""Summarise a rocprofv3 --stats kernel_stats.csv per train step (our kernels only)."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 13
OURS = ("gemm_", "reduce_splits", "composite", "sample_pdf", "stratified", "build_xd", "pe_xyz", "build_cin",
        "head_out", "geo_bwd", "transpose", "adam", "sqnorm", "rays_gen", "pick_pixels", "head_", "fused")
rows = list(csv.DictReader(open(path)))
tot = 0.0
out = []
for r in rows:
    if not any(k in r["Name"] for k in OURS):
        continue
    per = float(r["TotalDurationNs"]) / steps / 1e3
    tot += per
    out.append((per, int(r["Calls"]) / steps, float(r["AverageNs"]) / 1e3, r["Name"][:90]))
for per, c, avg, n in sorted(out, reverse=True):
    print(f"{per:9.1f} us/step  calls/step={c:5.1f}  avg={avg:8.1f} us  {n}")
print(f"sum of our kernels: {tot:.1f} us/step")
