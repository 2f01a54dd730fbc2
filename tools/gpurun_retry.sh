#!/bin/bash
# gpurun_retry.sh LOG TIMEOUT 'command': gpurun, retried only while nothing ran (exit 3: no free
# slot / box; status=transient: the box failed while being prepared, nothing charged); any other
# outcome ends the loop.
log=$1; to=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient.*run 0.0s" "$log"; then break; fi
  sleep 60
done
echo "rc=$rc tries=$i" >> "$log"
