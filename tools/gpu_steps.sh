#!/bin/bash
# Runs GPU steps in order, each under its own time limit.  Ordinary test
# failures (exit 1) let the next step run; a crash, abort or time limit
# (124, 134, 137, 139, or >128) ends the call there.
# usage: tools/gpu_steps.sh "<secs>|<name>|<command>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  secs=${spec%%|*}; rest=${spec#*|}; name=${rest%%|*}; cmd=${rest#*|}
  echo "== $name (limit ${secs}s)"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  tail -4 "gpurun_out/$name.log"
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -lt 0 ]; then echo "stopping after $name"; exit $rc; fi
done
