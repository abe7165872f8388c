set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bf16.py > gpurun_out/t_bf16.log 2>&1 || { tail -40 gpurun_out/t_bf16.log; exit 1; }
tail -1 gpurun_out/t_bf16.log
timeout -k 10 300 python tools/bench_mlp.py > gpurun_out/bm.log 2>&1 || { tail -30 gpurun_out/bm.log; exit 1; }
tail -1 gpurun_out/bm.log
