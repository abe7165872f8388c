set -o pipefail
cd /root/repo
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_streams.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_colpf.log 2>&1 || { tail -30 gpurun_out/pytest_colpf.log; exit 1; }
tail -1 gpurun_out/pytest_colpf.log
NERF_AMD_LIB=$PWD/exp/split1024.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_split1024.log 2>&1 || { tail -30 gpurun_out/pytest_split1024.log; exit 1; }
tail -1 gpurun_out/pytest_split1024.log
for rep in 1 2; do
for v in base split1024 split512; do
if [ $v = base ]; then L=""; else L="NERF_AMD_LIB=$PWD/exp/$v.so"; fi
env $L timeout -k 10 200 python bench.py --steps 30 --no-psnr --no-cpu-baseline --no-other-precision --no-dropin > gpurun_out/ab_$v$rep.log 2>&1 || { tail -20 gpurun_out/ab_$v$rep.log; exit 1; }
echo "split-ab rep $rep $v $(tail -1 gpurun_out/ab_$v$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["classes_ms"])')"
done; done
