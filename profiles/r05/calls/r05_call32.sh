#!/bin/bash
# Round 5, call 32: the default build with the raw-register bias sums (the A/B switch removed): bitwise against the
# measured variant exp/wbraw.so, all GPU tests on the default library, then the C2 A/B.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 120 python tools/lib_outputs.py --precision fp32 --out $O/def.pt > $O/lo_def.log 2>&1 || { tail $O/lo_def.log; exit 1; }
NERF_AMD_LIB=exp/wbraw.so timeout -k 10 120 python tools/lib_outputs.py --precision fp32 --out $O/wbraw.pt > $O/lo_wbraw.log 2>&1 || { tail $O/lo_wbraw.log; exit 1; }
python tools/lib_outputs.py --compare $O/def.pt $O/wbraw.pt || true; rm -f $O/*.pt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu_all.log 2>&1; tail -1 $O/pytest_gpu_all.log
cp nerf-sys_amd/lib/libnerf_amd.so exp/def.so
VARIANTS="def wbraw" ROUNDS=2 timeout -k 10 900 bash tools/ab_x6.sh
