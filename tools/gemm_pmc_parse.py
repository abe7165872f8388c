"""Per-kernel SQ / GRBM counters of a rocprofv3 --pmc run (tools/gemm_pmc.sh, tools/pmc_mfma_bench.sh): MFMA busy
fraction and effective clock per (kernel, grid).  MI355X_MICROARCH.md: SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed
over the SIMDs, GRBM_GUI_ACTIVE is summed over the 8 XCDs, so per dispatch clock = GRBM_GUI_ACTIVE / 8 / wall and MFMA
busy per SIMD = MFMA_BUSY / (256 CUs x 4 SIMDs x GRBM_GUI_ACTIVE / 8).  Wall times come from the counter collection's
own per-dispatch timestamps (profiled dispatches run serialised).  Usage: python tools/gemm_pmc_parse.py DIR"""
import collections
import csv
import glob
import statistics
import sys

root = sys.argv[1]
disp = collections.defaultdict(dict)
meta = {}
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d = r["Dispatch_Id"]
        disp[d][r["Counter_Name"]] = float(r["Counter_Value"])
        meta[d] = (r["Kernel_Name"][:70], r["Grid_Size"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
# persistent kernels launch the same grid for both nets: split a (kernel, grid) population at its largest wall-time
# gap when the longest dispatch is > 1.8x the shortest (the classes are then labelled by their median wall time)
groups = collections.defaultdict(list)
for d in disp:
    groups[meta[d][:2]].append(d)
label = {}
for key, ds in groups.items():
    ds.sort(key=lambda d: meta[d][2])
    ts = [meta[d][2] for d in ds]
    cut = len(ds)
    if len(ds) > 1 and ts[0] > 0 and ts[-1] / ts[0] > 1.8:
        cut = max(range(1, len(ds)), key=lambda i: ts[i] - ts[i - 1])
    for i, d in enumerate(ds):
        label[d] = "" if cut == len(ds) else ("short" if i < cut else "long")
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d, c in disp.items():
    name, grid, t = meta[d]
    grid = grid + (f" {label[d]}" if label[d] else "")
    g = c.get("GRBM_GUI_ACTIVE", 0.0)
    a = agg[(name, grid)]
    a["wall"].append(t)
    if t > 0 and g > 0:
        a["clock"].append(g / 8 / t / 1e9)
        a["busy"].append(c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024 * g / 8))
    if c.get("SQ_WAVE_CYCLES"):
        a["wait"].append(c.get("SQ_WAIT_ANY", 0.0) / c["SQ_WAVE_CYCLES"])
        for k, n in (("SQ_WAIT_INST_ANY", "winst"), ("SQ_ACTIVE_INST_ANY", "active"), ("SQ_WAIT_INST_LDS", "wlds")):
            if k in c:
                a[n].append(c[k] / c["SQ_WAVE_CYCLES"])
    a["lds"].append(c.get("SQ_LDS_BANK_CONFLICT", 0.0))
med = lambda xs: statistics.median(xs) if xs else float("nan")
for (name, grid), a in sorted(agg.items()):
    print(f"{name:70s} grid {grid:>15s} n {len(a['wall']):3d}  wall {med(a['wall']) * 1e3:7.3f} ms  clock {med(a['clock']):5.2f} GHz  "
          f"MFMA busy {med(a['busy']):5.3f}  waits/wave-cycles {med(a['wait']):5.3f}  LDS conflicts {med(a['lds']):.3g}" +
          (f"  issue-stall {med(a['winst']):5.3f}  active {med(a['active']):5.3f}  lds-issue-stall {med(a['wlds']):5.3f}"
           if a["winst"] else ""))
