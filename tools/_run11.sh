set -o pipefail
cd /root/repo
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_streams.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_x6b.log 2>&1 || { tail -30 gpurun_out/pytest_x6b.log; exit 1; }
tail -1 gpurun_out/pytest_x6b.log
timeout -k 10 300 python bench.py --steps 30 --no-psnr --no-cpu-baseline --no-other-precision --no-dropin > gpurun_out/bench_x6b.log 2>&1 || { tail -20 gpurun_out/bench_x6b.log; exit 1; }
tail -1 gpurun_out/bench_x6b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("split", d["value"], d["ms_per_step"], d["roofline"]["classes_ms"]); print("native", d["fp32_native_gemm"])'
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_x6b -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-psnr --no-dropin --no-other-precision --no-native-ref > gpurun_out/prof_x6b.log 2>&1 || { tail -20 gpurun_out/prof_x6b.log; exit 1; }
python3 tools/step_timeline.py gpurun_out/prof_x6b/run_kernel_trace.csv > gpurun_out/step_x6b.txt 2>&1 || true
sed -n 18,32p gpurun_out/step_x6b.txt | cut -c1-120; sed -n 33,50p gpurun_out/step_x6b.txt | cut -c1-120
