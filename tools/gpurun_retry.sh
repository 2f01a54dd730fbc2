#!/bin/bash
# gpurun_retry.sh LOG TIMEOUT 'command': gpurun, retried only while it reports no free slot / box
# (exit 3: nothing ran, nothing charged); any other outcome ends the loop.
log=$1; to=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  sleep 150
done
echo "rc=$rc tries=$i" >> "$log"
