#!/bin/bash
# (development helper, not run on the GPU box)
# retry gpurun only while the pool has no box/slot (infrastructure status, nothing ran); usage: gpr.sh LOG TIMEOUT CMD
log=$1; to=$2; shift 2
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $log 2>&1
  rc=$?
  if grep -q "status=transient" $log && ! grep -q "run [1-9]" $log; then sleep 90; continue; fi
  break
done
tail -15 $log
