#!/bin/bash
# rocprofv3 passes for the bench workloads (run on the GPU box from the repo root). Each
# workload is profiled on its own, so a kernel's per-dispatch average belongs to one config:
#   p361: the headline layer step (P = 361), p190: the side-line layer step (P = 190),
#   rest: KLD step, push, k-NN, eval, bound boxes (P = 190).
# Per workload: 1. --kernel-trace --stats  2. --pmc FETCH_SIZE  3. --pmc WRITE_SIZE (own passes;
# counters never share a pass with tracing domains other than the kernel trace).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r03}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
# one configuration per workload: no side lines that launch the same kernels at other shapes
B=(python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-small-batch --no-train --no-sigmoid)
declare -A ARGS
ARGS[p361]="--protos 361 --side-protos 0 --no-kld --no-push --no-knn --no-eval --no-wide"
ARGS[p190]="--protos 190 --side-protos 0 --no-kld --no-push --no-knn --no-eval --no-wide"
ARGS[rest]="--protos 190 --side-protos 0"
run() {  # run <workload> <pass> <seconds> <rocprof args...>
  local wl=$1 name=$2 secs=$3; shift 3
  echo "== $wl/$name ($(date +%T))"
  # shellcheck disable=SC2086
  timeout -k 10 "$secs" rocprofv3 "$@" -d "$OUT/$wl/$name" -o "$name" --output-format csv -- "${B[@]}" ${ARGS[$wl]} \
    > "$OUT/$wl/$name.log" 2>&1
  local rc=$?
  echo "== $wl/$name rc=$rc"; tail -n 1 "$OUT/$wl/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
for wl in ${WORKLOADS:-p361 p190 rest}; do
  mkdir -p "$OUT/$wl"
  run "$wl" trace 300 --kernel-trace --stats -T
  run "$wl" fetch 300 --kernel-trace --pmc FETCH_SIZE -T
  run "$wl" write 300 --kernel-trace --pmc WRITE_SIZE -T
done
