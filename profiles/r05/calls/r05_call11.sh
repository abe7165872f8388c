#!/bin/bash
# Round 5, call 11: (1) the engine probe under the SQ set with counters collected only on the two dominant bf16
# kernels (--kernel-include-regex), 8000 steps; (2) the unfiltered one-stream probe again with the runtime libraries'
# base addresses printed, so the crash PCs map to a library + offset.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
timeout -s KILL 500 rocprofv3 --pmc $SQ --kernel-include-regex "bwd_layer|mlp_fwd_fused" --kernel-trace --output-format csv -d $O/eprobe5 -o run -- \
  python3 tools/pmc_engine_probe.py --precision bf16 --steps 8000 --every 250 > $O/eprobe5.log 2>&1
rc=$?; echo "engine probe 8000, counters on 2 kernels: rc=$rc"; grep -v "^W20\|^E20" $O/eprobe5.log | grep -E "probe|Fatal|SIGSEGV|File" | tail -4
ls -la $O/eprobe5/*/ 2>/dev/null | head; python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/r05/eprobe5/**/*counter_collection.csv", recursive=True):
    n = set(); k = {}
    for r in csv.DictReader(open(f)):
        n.add(r.get("Dispatch_Id")); k[r.get("Kernel_Name", "")[:60]] = k.get(r.get("Kernel_Name", "")[:60], 0) + 1
    print(f, "dispatches with counters:", len(n)); [print("  ", v, kk) for kk, v in sorted(k.items())[:6]]
PY
rm -rf $O/eprobe5/*.csv $O/eprobe5/*/*.csv 2>/dev/null
[ $rc -ne 0 ] && exit 0
timeout -s KILL 400 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d $O/eprobe6 -o run -- \
  python3 tools/pmc_engine_probe.py --precision bf16 --steps 3000 --every 100 --no-overlap > $O/eprobe6.log 2>&1
rc=$?; echo "engine probe 3000, one stream, all counted: rc=$rc"; grep -v "^W20\|^E20" $O/eprobe6.log | grep -E "probe|Fatal|SIGSEGV|File" | tail -14
rm -rf $O/eprobe6/*.csv $O/eprobe6/*/*.csv 2>/dev/null
exit 0
