set -o pipefail
mkdir -p gpurun_out/bf
timeout -k 10 200 ./tools/gemm_bf16_test > gpurun_out/bf/gemm_bf16_test.log 2>&1; rc=$?; grep -E "wsr|OK|FAIL" gpurun_out/bf/gemm_bf16_test.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 600 python -m pytest tests/test_gpu_bf16.py -q -x > gpurun_out/bf/pytest_bf16.log 2>&1; rc=$?; tail -3 gpurun_out/bf/pytest_bf16.log; [[ $rc -ne 0 ]] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --precision bf16 > gpurun_out/bf/bench_bf16.log 2>&1 || exit 1
tail -1 gpurun_out/bf/bench_bf16.log | cut -c1-200
