set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
for o in fwd bwd; do
NERF_OVERLAP=$o timeout -k 10 300 python bench.py --precision bf16 --no-cpu-baseline --no-psnr > gpurun_out/b_$o.log 2>&1 || { tail -30 gpurun_out/b_$o.log; exit 1; }
echo $o; tail -1 gpurun_out/b_$o.log | cut -c1-200
done
NERF_OVERLAP=bwd timeout -k 10 300 python bench.py --no-cpu-baseline --no-psnr --no-dropin > gpurun_out/b_f32.log 2>&1 || { tail -30 gpurun_out/b_f32.log; exit 1; }
echo fp32-bwd; tail -1 gpurun_out/b_f32.log | cut -c1-200
