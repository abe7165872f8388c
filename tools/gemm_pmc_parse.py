"""Per-kernel SQ / GRBM counters of tools/gemm_pmc.sh runs: MFMA busy fraction and the effective clock.
MI355X_MICROARCH.md: SQ_VALU_MFMA_BUSY_CYCLES counts cycles (summed over SIMDs), GRBM_GUI_ACTIVE is summed over the
8 XCDs, so clock = GRBM_GUI_ACTIVE / 8 / kernel wall time; MFMA busy per SIMD = MFMA_BUSY / (256 CUs x 4 SIMDs x
GRBM_GUI_ACTIVE / 8).  Usage: python tools/gemm_pmc_parse.py gpurun_out/gpmc/p1"""
import collections
import csv
import glob
import sys

root = sys.argv[1]
ctr = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        key = (r["Kernel_Name"][:70], r.get("Grid_Size", ""))
        ctr[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = collections.defaultdict(list)
for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Kernel_Name"][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
for (name, grid), d in sorted(ctr.items()):
    m = {k: sum(v) / len(v) for k, v in d.items()}
    ts = dur.get(name)
    t = sorted(ts)[len(ts) // 2] if ts else float("nan")
    clk = m.get("GRBM_GUI_ACTIVE", 0) / 8 / t / 1e9 if ts else float("nan")
    busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (1024 * m.get("GRBM_GUI_ACTIVE", 1) / 8)
    print(f"{name:70s} grid {grid:>9s} wall {t * 1e3:7.3f} ms  clock {clk:5.2f} GHz  MFMA busy {busy:5.3f}  "
          f"waits/wave-cycles {m.get('SQ_WAIT_ANY', 0) / max(m.get('SQ_WAVE_CYCLES', 1), 1):5.3f}  "
          f"LDS conflicts {m.get('SQ_LDS_BANK_CONFLICT', 0):.3g}")
