#!/bin/bash
# usage: scripts/gpr.sh LOG TIMEOUT 'cmd'  -- retries only while no GPU slot/box is free (rc 3: nothing ran, nothing charged)
log=$1; to=$2; shift 2
for i in $(seq 1 30); do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $log 2>&1
  rc=$?
  echo "[gpr] attempt $i rc=$rc" >> $log
  if [ $rc -ne 3 ]; then exit $rc; fi
  sleep 90
done
