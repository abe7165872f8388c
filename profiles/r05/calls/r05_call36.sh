#!/bin/bash
# Round 5, call 36: the narrow weight gradient (gemm_wgrad_x6_kernel, four register sets) with whole rounds in the
# loop and the partial round peeled (its latch drained all 12 loads in flight every four slabs): bitwise check against
# the HEAD build exp/def.so, all GPU tests on the in-tree build (= exp/npeel.so), then the C2 A/B.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
for v in def npeel; do
  NERF_AMD_LIB=exp/$v.so timeout -k 10 120 python tools/lib_outputs.py --precision fp32 --out $O/$v.pt > $O/lo_$v.log 2>&1 || { tail $O/lo_$v.log; exit 1; }
done
python tools/lib_outputs.py --compare $O/npeel.pt $O/def.pt || true; rm -f $O/*.pt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu_all.log 2>&1; tail -1 $O/pytest_gpu_all.log
VARIANTS="def npeel" ROUNDS=3 timeout -k 10 900 bash tools/ab_x6.sh
