set -o pipefail
cd /root/repo
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_x6.log 2>&1 || { tail -20 gpurun_out/smoke_x6.log; exit 1; }
tail -1 gpurun_out/smoke_x6.log
for v in split split_dgrad; do
timeout -k 10 200 python bench.py --steps 20 --no-psnr --no-cpu-baseline --no-other-precision --no-dropin --fp32-gemm $v > gpurun_out/ab_g_$v.log 2>&1 || { tail -20 gpurun_out/ab_g_$v.log; exit 1; }
echo "gemm-ab $v $(tail -1 gpurun_out/ab_g_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["classes_ms"], r["classes_engine"], r["class"], r["achieved"], r["frac"], "native", d["fp32_native_gemm"]["value"])')"
done
