#!/bin/bash
# device-sized container step: its GPU tests, the bench line in both modes (alternated), a kernel-trace timeline
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06/$1; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_moe.py tests/test_gpu_occ.py -x -q --timeout 120 --timeout-method thread > $O/pytest_moe.log 2>&1 || { tail -40 $O/pytest_moe.log; exit 1; }
tail -1 $O/pytest_moe.log
for mode in dev host dev host; do
  F=""; [ $mode = host ] && F="--host-sized"
  timeout -k 10 300 python tools/bench_container.py --no-cpu-baseline --steps 48 --warmup 40 $F > $O/bc_$mode.log 2>&1 || { tail -30 $O/bc_$mode.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/bc_$mode.log').read().strip().splitlines()[-1]); print('$mode', d['value'], d['ms_per_step'], d['kernels_ms_per_step'], d['samples_per_step'], d.get('device_sized'))"
done
[ -n "$NO_PROF" ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cont -o run --output-format csv -- python3 tools/bench_container.py --no-cpu-baseline --steps 48 --warmup 40 > $O/prof_cont.log 2>&1 || { tail -20 $O/prof_cont.log; exit 1; }
python3 tools/cont_timeline.py $O/prof_cont/run_kernel_trace.csv 60 48 > $O/step_cont.txt 2>&1 || true
rm -f $O/prof_cont/run_kernel_trace.csv
tail -4 $O/step_cont.txt
