set -o pipefail
cd /root/repo
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -Wno-unused-result tools/stream_probe.hip -o /tmp/stream_probe > /dev/null 2>&1 || echo "probe build failed"
timeout -k 10 60 /tmp/stream_probe 2>&1 | tee gpurun_out/stream_probe.txt || exit 1
VARIANTS="base fwd_NOMFMA fwd_NOWLOAD fwd_NOEPI fwd_NOSTORE fwd_ONLYMFMA" bash tools/exp_bwd.sh 2>&1 | tee gpurun_out/exp_fwd.txt
