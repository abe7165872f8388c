set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
for v in s4096 s8192; do
NERF_AMD_LIB=$PWD/exp/$v.so timeout -k 10 300 python tools/bench_mlp.py > gpurun_out/bm_$v.log 2>&1 || { tail -30 gpurun_out/bm_$v.log; exit 1; }
echo $v; tail -1 gpurun_out/bm_$v.log
NERF_AMD_LIB=$PWD/exp/$v.so timeout -k 10 300 python tools/bench_mlp.py --M 262144 > gpurun_out/bm_$v.log 2>&1 || { tail -30 gpurun_out/bm_$v.log; exit 1; }
tail -1 gpurun_out/bm_$v.log
done
timeout -k 10 300 python tools/bench_mlp.py --M 262144 > gpurun_out/bm_c.log 2>&1 || { tail -30 gpurun_out/bm_c.log; exit 1; }
tail -1 gpurun_out/bm_c.log
