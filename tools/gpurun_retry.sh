#!/bin/bash
# usage: gpr.sh LOG TIMEOUT CMD  -- retries gpurun only while no box/slot is free (rc 3)
log=$1; to=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$log"; then echo "rc=$rc" >> "$log"; exit $rc; fi
  if [ $rc -ne 3 ] && grep -q "status=transient" "$log" && grep -q "run [1-9]" "$log"; then echo "rc=$rc" >> "$log"; exit $rc; fi
  sleep 100
done
