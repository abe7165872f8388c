set -o pipefail
cd /root/repo
for v in base x6bk16m3 base x6bk16m3; do
if [ $v = base ]; then L=""; else L="NERF_AMD_LIB=$PWD/exp/$v.so"; fi
env $L timeout -k 10 200 python bench.py --steps 20 --no-psnr --no-cpu-baseline --no-other-precision --no-dropin --no-native-ref > gpurun_out/abl_$v.log 2>&1 || { tail -20 gpurun_out/abl_$v.log; exit 1; }
echo "x6-ab $v $(tail -1 gpurun_out/abl_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["classes_ms"])')"
done
