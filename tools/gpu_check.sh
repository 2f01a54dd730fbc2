#!/bin/bash
# GPU validation pass for the box: smoke -> gpu tests -> short bench. Every GPU step has its
# own time limit; a crash / abort / timeout (anything but a plain test failure, exit 1) stops
# the script so nothing else touches the GPU after a fault.
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 25 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "== stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step smoke 400 python __graft_entry__.py smoke
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:randomly --timeout 120 --timeout-method thread
step bench 600 python bench.py --steps 20 --warmup 5 --cpu-seconds 8
