set -o pipefail
cd /root/repo
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_all_x6.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_all_x6.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_all_x6.log
PMC_OUT=gpurun_out/pmc_x6t PMC_BENCH_ARGS="--no-dropin --no-other-precision --no-native-ref" bash tools/pmc_traffic.sh > gpurun_out/pmc_x6t.txt 2>&1 || { tail -20 gpurun_out/pmc_x6t.txt; exit 1; }
tail -3 gpurun_out/pmc_x6t.txt
