#!/bin/bash
# Round 5, call 9: rocprofv3 --pmc dispatch limit.  The engine probe died between 5500 and 5750 bf16 steps (call 8);
# here N torch dispatches with no code of this repository: (1) 300k under the SQ set; (2) 300k with
# --kernel-include-regex matching no kernel (counters collected on none of them).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
timeout -s KILL 300 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d $O/dprobe1 -o run -- \
  python3 tools/pmc_dispatch_probe.py --n 300000 --every 2000 > $O/dprobe1.log 2>&1
rc=$?; echo "dispatch probe 300k, all dispatches counted: rc=$rc"; grep -v "^W20\|^E20" $O/dprobe1.log | grep -E "probe|Fatal|SIGSEGV" | tail -3
rm -rf $O/dprobe1/*.csv $O/dprobe1/*/*.csv 2>/dev/null
[ $rc -ne 0 ] && [ $rc -ne 139 ] && exit 0
timeout -s KILL 300 rocprofv3 --pmc $SQ --kernel-include-regex "no_kernel_has_this_name" --kernel-trace --output-format csv -d $O/dprobe2 -o run -- \
  python3 tools/pmc_dispatch_probe.py --n 300000 --every 2000 > $O/dprobe2.log 2>&1
rc=$?; echo "dispatch probe 300k, no dispatch counted: rc=$rc"; grep -v "^W20\|^E20" $O/dprobe2.log | grep -E "probe|Fatal|SIGSEGV" | tail -3
rm -rf $O/dprobe2/*.csv $O/dprobe2/*/*.csv 2>/dev/null
exit 0
