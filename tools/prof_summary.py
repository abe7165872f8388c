"""Summarise a rocprofv3 --stats kernel_stats.csv per train step (our kernels only).

  python tools/prof_summary.py run_kernel_stats.csv STEPS [ROOFLINE_STEPS]

STEPS = engine steps in the profiled run (warmup + timed + roofline pass); ROOFLINE_STEPS (bench.py --timing-steps,
default 3) = the isolated steps bench.py runs after its timed region for the live roofline: the per-(kernel, grid)
table then also averages only each population's launches of those last steps — the launches the bench line's
`roofline.mean_launch_ms` is measured on."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 13
OURS = ("gemm_", "reduce_splits", "composite", "sample_pdf", "stratified", "build_xd", "pe_xyz", "build_cin",
        "head_out", "geo_bwd", "transpose", "adam", "sqnorm", "rays_gen", "pick_pixels", "head_", "fused",
        "bwd_layer", "bwd_tail", "reduce_fused", "pe_prefill", "frag_pack", "color_bwd", "fwd_tail", "x6_planes")
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


# per (kernel, grid) averages from the kernel trace next to the stats file: the roofline kernel's launches
# are told apart from other launches of the same symbol by their grid (fine net trunk: M = 786,432 rows)
import glob
import os
tr = glob.glob(os.path.join(os.path.dirname(path), "*kernel_trace.csv"))
if tr:
    from collections import defaultdict
    per = defaultdict(list)
    for r in csv.DictReader(open(tr[0])):
        if not r["Kernel_Name"].startswith("void gemm_"):
            continue
        blocks = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
        per[(r["Kernel_Name"].split("(")[0], blocks)].append(
            (int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    rsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    print("\nper (GEMM kernel, grid) launch averages from the kernel trace (all launches | the launches of the last "
          f"{rsteps} steps = bench.py's isolated roofline pass):")
    for (n, b), v in sorted(per.items(), key=lambda kv: -sum(d for _, d in kv[1])):
        v.sort()
        k = max(1, round(len(v) * rsteps / steps))
        tail = [d for _, d in v[-k:]]
        allv = [d for _, d in v]
        print(f"{sum(allv) / len(allv):9.1f} us avg x{len(allv):4d} | {sum(tail) / len(tail):9.1f} us avg x{k:3d}  "
              f"blocks={b:6d}  {n[:80]}")
