#!/bin/bash
# End-of-round check as the driver runs it: smoke, every GPU test, then bench.py with defaults.
set -u
OUT=${OUT:-gpurun_out/final}
mkdir -p "$OUT"
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 4 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step smoke 400 python __graft_entry__.py smoke
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench 900 python bench.py
