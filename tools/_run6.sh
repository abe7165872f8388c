set -o pipefail
cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_streams.py tests/test_gpu_dropin.py tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_tail.log 2>&1 || { tail -40 gpurun_out/pytest_tail.log; exit 1; }
tail -2 gpurun_out/pytest_tail.log
for rep in 1 2; do
for v in base tailchain; do
if [ $v = base ]; then L=""; else L="NERF_AMD_LIB=$PWD/exp/$v.so"; fi
env $L timeout -k 10 200 python bench.py --steps 30 --no-psnr --no-cpu-baseline --no-other-precision --no-dropin > gpurun_out/ab_$v$rep.log 2>&1 || { tail -20 gpurun_out/ab_$v$rep.log; exit 1; }
echo "tail-ab rep $rep $v $(tail -1 gpurun_out/ab_$v$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["class"], d["roofline"]["mean_launch_ms"])')"
done; done
