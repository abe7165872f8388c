set -o pipefail
cd /root/repo
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_x6_parity.log 2>&1 || { grep -E "PASS|FAIL|Error|error" gpurun_out/pytest_x6_parity.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_x6_parity.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_streams.py tests/test_gpu_edges.py tests/test_gpu_dropin.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_x6_more.log 2>&1 || { tail -30 gpurun_out/pytest_x6_more.log; exit 1; }
tail -1 gpurun_out/pytest_x6_more.log
timeout -k 10 300 python bench.py --steps 30 --no-psnr --no-cpu-baseline --no-other-precision --no-dropin > gpurun_out/bench_x6.log 2>&1 || { tail -20 gpurun_out/bench_x6.log; exit 1; }
tail -1 gpurun_out/bench_x6.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("split", d["value"], d["ms_per_step"], d["roofline"]["classes_ms"]); print("native", d["fp32_native_gemm"])'
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_x6 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-psnr --no-dropin --no-other-precision --no-native-ref > gpurun_out/prof_x6.log 2>&1 || { tail -20 gpurun_out/prof_x6.log; exit 1; }
python3 tools/step_timeline.py gpurun_out/prof_x6/run_kernel_trace.csv > gpurun_out/step_x6.txt 2>&1 || true
head -60 gpurun_out/step_x6.txt | cut -c1-140
