set -o pipefail
cd /root/repo
NERF_AMD_LIB=$PWD/exp/bigsmall.so timeout -k 10 400 python -u -m pytest tests/test_gpu_split_gemm.py -x -q -s --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_bigsmall.log 2>&1 || { tail -30 gpurun_out/pytest_bigsmall.log; exit 1; }
grep "M=262144" gpurun_out/pytest_bigsmall.log | head -16; tail -1 gpurun_out/pytest_bigsmall.log
for v in "base split" "bigsmall split_dgrad" "base split_dgrad"; do
set -- $v
if [ $1 = base ]; then L=""; else L="NERF_AMD_LIB=$PWD/exp/$1.so"; fi
env $L timeout -k 10 200 python bench.py --steps 20 --no-psnr --no-cpu-baseline --no-other-precision --no-dropin --no-native-ref --fp32-gemm $2 > gpurun_out/abl_$1_$2.log 2>&1 || { tail -20 gpurun_out/abl_$1_$2.log; exit 1; }
echo "x6-ab $1 $2 $(tail -1 gpurun_out/abl_$1_$2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["classes_ms"])')"
done
