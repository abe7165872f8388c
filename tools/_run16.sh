set -o pipefail
cd /root/repo
NERF_AMD_LIB=$PWD/exp/x6pipe.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split_gemm.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_x6pipe.log 2>&1 || { tail -30 gpurun_out/pytest_x6pipe.log; exit 1; }
tail -1 gpurun_out/pytest_x6pipe.log
for v in base x6pipe base x6pipe; do
if [ $v = base ]; then L=""; else L="NERF_AMD_LIB=$PWD/exp/$v.so"; fi
env $L timeout -k 10 200 python bench.py --steps 20 --no-psnr --no-cpu-baseline --no-other-precision --no-dropin --no-native-ref > gpurun_out/abl_$v.log 2>&1 || { tail -20 gpurun_out/abl_$v.log; exit 1; }
echo "x6-ab $v $(tail -1 gpurun_out/abl_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["classes_ms"])')"
done
