set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_convergence.py > gpurun_out/t_conv.log 2>&1 || { tail -40 gpurun_out/t_conv.log; exit 1; }
grep -E "PASS|FAIL|passed|failed|matched" gpurun_out/t_conv.log | tail -5
