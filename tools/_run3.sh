set -o pipefail
cd /root/repo
VARIANTS="base bwd_NOIO bwd_NOWG bwd_NODG bwd_NOSTORE bwd_NOMFMA bwd_IOONLY" bash tools/exp_bwd.sh 2>&1 | tee gpurun_out/exp_bwd.txt || exit 1
TESTS=tests/test_gpu_dp.py bash tools/r03_check.sh
