#!/bin/bash
# gpurun with a retry when no GPU slot / box is free (exit 3, or a transient box-preparation failure; nothing was
# charged in either case).  Usage: tools/gpu_call.sh OUTFILE TIMEOUT 'command'
out=$1; to=$2; shift 2
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$out" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$out"; then sleep 100; continue; fi
  exit $rc
done
exit $rc
