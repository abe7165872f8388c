#!/bin/bash
# Round 5, call 10: is the rocprofv3 --pmc failure tied to launches from two HIP streams?  (1) the engine probe with
# no side stream, 8000 bf16 steps (the two-stream run died after 5500); (2) 300k torch dispatches alternating over
# two streams.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
timeout -s KILL 500 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d $O/eprobe4 -o run -- \
  python3 tools/pmc_engine_probe.py --precision bf16 --steps 8000 --every 250 --no-overlap > $O/eprobe4.log 2>&1
rc=$?; echo "engine probe 8000, one stream: rc=$rc"; grep -v "^W20\|^E20" $O/eprobe4.log | grep -E "probe|Fatal|SIGSEGV|File" | tail -4
rm -rf $O/eprobe4/*.csv $O/eprobe4/*/*.csv 2>/dev/null
[ $rc -ne 0 ] && exit 0
timeout -s KILL 300 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d $O/dprobe3 -o run -- \
  python3 tools/pmc_dispatch_probe.py --n 300000 --every 2000 --streams 2 > $O/dprobe3.log 2>&1
rc=$?; echo "dispatch probe 300k over 2 streams: rc=$rc"; grep -v "^W20\|^E20" $O/dprobe3.log | grep -E "probe|Fatal|SIGSEGV|File" | tail -4
rm -rf $O/dprobe3/*.csv $O/dprobe3/*/*.csv 2>/dev/null
exit 0
