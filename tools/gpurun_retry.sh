#!/bin/bash
# usage: gpurun_retry.sh LOG TIMEOUT CMD -- runs gpurun, again only while no box/slot was free
# (exit 3 or a "transient" verdict: nothing ran, nothing was charged); any run that started is
# never repeated
log=$1; to=$2; shift 2
for i in $(seq 1 30); do
  rm -f gpurun_out/.last_call.json
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ $rc -ne 3 ] && [ "$st" != "transient" ]; then echo "rc=$rc" >> "$log"; exit $rc; fi
  sleep 90
done
exit 3
