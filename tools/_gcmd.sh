# quick GPU check used during development: NGP / MoE / occupancy / meta tests, then the NGP and container benches
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ngp.py tests/test_gpu_moe.py tests/test_gpu_occ.py tests/test_gpu_meta.py > gpurun_out/t1.log 2>&1 || { tail -40 gpurun_out/t1.log; exit 1; }
tail -1 gpurun_out/t1.log
timeout -k 10 300 python3 tools/bench_ngp.py --no-cpu-baseline > gpurun_out/bn.log 2>&1 || { tail -20 gpurun_out/bn.log; exit 1; }
tail -1 gpurun_out/bn.log | cut -c1-650
timeout -k 10 300 python3 tools/bench_container.py --steps 20 --warmup 40 --no-cpu-baseline > gpurun_out/bc.log 2>&1 || { tail -20 gpurun_out/bc.log; exit 1; }
tail -1 gpurun_out/bc.log | cut -c1-700
