set -o pipefail
cd /root/repo
timeout -k 10 300 python -u -m pytest tests/test_gpu_streams.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_streams.log 2>&1 || { tail -30 gpurun_out/pytest_streams.log; exit 1; }
tail -2 gpurun_out/pytest_streams.log
for rep in 1 2; do
for f in "" "--no-split-wgrad"; do
timeout -k 10 200 python bench.py --steps 30 --no-psnr --no-cpu-baseline --no-other-precision --no-dropin $f > gpurun_out/ab_split$rep$f.log 2>&1 || { tail -20 gpurun_out/ab_split$rep$f.log; exit 1; }
echo "split-ab rep $rep [$f] $(tail -1 gpurun_out/ab_split$rep$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["class"], d["roofline"]["mean_launch_ms"], d["roofline"]["classes_ms"])')"
done; done
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/stream_probe.hip -o /tmp/stream_probe > /dev/null 2>&1 || echo "probe build failed"
timeout -k 10 120 /tmp/stream_probe 2>&1 | tee gpurun_out/stream_probe.txt || exit 1
VARIANTS="base fwd_NOMFMA fwd_NOWLOAD fwd_NOEPI fwd_NOSTORE fwd_ONLYMFMA" bash tools/exp_bwd.sh 2>&1 | tee gpurun_out/exp_fwd.txt
