#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box from the repo root):
#   1. --kernel-trace --stats          -> per-kernel average durations
#   2. --pmc FETCH_SIZE (own pass)     -> HBM read bytes per dispatch
#   3. --pmc WRITE_SIZE (own pass)     -> HBM write bytes per dispatch
# Counters never share a pass with tracing domains other than the kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r01}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH=(python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline)
run() {  # run <name> <seconds> <rocprof args...>
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" rocprofv3 "$@" -d "$OUT/$name" -o "$name" --output-format csv -- "${BENCH[@]}" \
    > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run trace 600 --kernel-trace --stats -T
run fetch 600 --kernel-trace --pmc FETCH_SIZE -T
run write 600 --kernel-trace --pmc WRITE_SIZE -T
find "$OUT" -name "*.csv" | head -20
