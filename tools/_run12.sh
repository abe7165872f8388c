set -o pipefail
cd /root/repo
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_streams.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_x6w.log 2>&1 || { tail -30 gpurun_out/pytest_x6w.log; exit 1; }
tail -1 gpurun_out/pytest_x6w.log
for v in base x6square base; do
if [ $v = base ]; then L=""; else L="NERF_AMD_LIB=$PWD/exp/$v.so"; fi
env $L timeout -k 10 200 python bench.py --steps 20 --no-psnr --no-cpu-baseline --no-other-precision --no-dropin --no-native-ref > gpurun_out/abl_$v.log 2>&1 || { tail -20 gpurun_out/abl_$v.log; exit 1; }
echo "x6-ab $v $(tail -1 gpurun_out/abl_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["classes_ms"])')"
done
PMC_OUT=gpurun_out/pmc_x6w PMC_BENCH_ARGS="--no-other-precision --no-native-ref" bash tools/pmc_mfma_bench.sh > /dev/null 2>&1 || exit 1
grep "x6" gpurun_out/pmc_x6w/summary.txt | cut -c1-230
