#!/bin/bash
# gpurun, retried only while the pool has no box free (exit 3: nothing ran,
# nothing charged); any other outcome is returned as is.
#   tools/gpurun_wait.sh OUTFILE TIMEOUT 'command'
out=$1; lim=$2; shift 2
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$@" > "$out" 2>&1
  rc=$?
  [ $rc -ne 3 ] && ! grep -q "no free box right now\|backing off\|status=transient" "$out" && exit $rc
  sleep 90
done
exit $rc
