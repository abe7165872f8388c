set -o pipefail
cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_gpu_split_gemm.py tests/test_gpu_parity.py tests/test_gpu_streams.py tests/test_gpu_edges.py tests/test_gpu_dropin.py -x -q -s --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_bs.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/pytest_bs.log | tail -30; exit 1; }
grep "M=262144 tensor" gpurun_out/pytest_bs.log | head -16; tail -1 gpurun_out/pytest_bs.log
for v in split native_dgrad; do
timeout -k 10 200 python bench.py --steps 20 --no-psnr --no-cpu-baseline --no-other-precision --no-dropin --fp32-gemm $v > gpurun_out/ab_bs_$v.log 2>&1 || { tail -20 gpurun_out/ab_bs_$v.log; exit 1; }
echo "gemm-ab $v $(tail -1 gpurun_out/ab_bs_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["classes_ms"], r["class"], r["frac"], "native", d["fp32_native_gemm"]["value"])')"
done
