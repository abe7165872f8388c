#!/bin/bash
# Round 5, call 22: the fp16 epilogue on v_fma_mix_f32 (default build) vs the widening form (exp/nomix.so): bitwise
# outputs, fp16 tests on the default build, then the AMP loop A/B (tools/amp_kernels_ab.py) on both builds.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
NERF_AMD_LIB=exp/mix.so timeout -k 10 120 python tools/lib_outputs.py --precision fp16 --out $O/mix.pt > $O/lo_mix.log 2>&1 || { tail $O/lo_mix.log; exit 1; }
NERF_AMD_LIB=exp/nomix.so timeout -k 10 120 python tools/lib_outputs.py --precision fp16 --out $O/nomix.pt > $O/lo_nomix.log 2>&1 || { tail $O/lo_nomix.log; exit 1; }
python tools/lib_outputs.py --compare $O/mix.pt $O/nomix.pt; rm -f $O/mix.pt $O/nomix.pt
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp16.py tests/test_gpu_dropin.py -m gpu -q --timeout 240 --timeout-method thread > $O/pytest_c22.log 2>&1; rc=$?; tail -2 $O/pytest_c22.log
[ $rc -ne 0 ] && exit 1
for r in 1 2; do for v in nomix mix; do
  NERF_AMD_LIB=exp/$v.so timeout -k 10 300 python3 tools/amp_kernels_ab.py > $O/amp_$v.log 2>&1 || { tail $O/amp_$v.log; exit 1; }
  echo "$v: $(grep -E '^fp16 ' $O/amp_$v.log | cut -c1-80) | $(grep -E '^bf16 ' $O/amp_$v.log | cut -c1-80)"
done; done
