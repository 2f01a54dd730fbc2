#!/bin/bash
# usage: bash tools/gpu_run.sh TAG STEP...  — each STEP is "name:timeout:command"; runs the steps in
# order under their own time limits, logs to gpurun_out/TAG_name.log, stops at the first failure.
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
for step in "$@"; do
  name=${step%%:*}; rest=${step#*:}; to=${rest%%:*}; cmd=${rest#*:}
  echo "== $name ($to s): $cmd"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/${tag}_${name}.log" 2>&1
  rc=$?
  tail -4 "gpurun_out/${tag}_${name}.log"
  if [ $rc -ne 0 ]; then echo "!! $name failed rc=$rc"; exit $rc; fi
done
