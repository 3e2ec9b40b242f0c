#!/bin/bash
# (development helper, not run on the GPU box)
# retry gpurun only while the pool has no box/slot (infrastructure status, nothing ran), waiting as long as
# gpurun asks; usage: gpr.sh LOG TIMEOUT CMD
log=$1; to=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $log 2>&1
  if grep -q "status=transient" $log && ! grep -q "run [1-9]" $log; then
    w=$(grep -o "retry in [0-9]*s" $log | grep -o "[0-9]*" | tail -1)
    sleep $(( ${w:-90} + 15 ))
    continue
  fi
  break
done
tail -15 $log
