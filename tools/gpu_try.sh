#!/bin/bash
# usage: gpu_try.sh OUTFILE TIMEOUT 'command'   — retries ONLY when the call never ran (transient / no slot)
out=$1; to=$2; cmd=$3
for i in 1 2 3 4 5 6 7 8 9 10 11 12; do
  /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $out 2>&1
  rc=$?
  if grep -q "status=transient\|no free box\|slot(s) on this pod are busy\|backing off" $out && ! grep -q "status=ok\|status=fail" $out; then
    sleep 90; continue
  fi
  exit $rc
done
