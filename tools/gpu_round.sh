#!/bin/bash
# Round check: smoke + all GPU tests + bench (tools/gpu_check.sh), then the rocprofv3 passes of
# every bench workload (tools/profile.sh: kernel stats + FETCH_SIZE + WRITE_SIZE).
set -u
OUT=${OUT:-gpurun_out/round}
mkdir -p "$OUT"
OUT=$OUT bash tools/gpu_check.sh || exit $?
grep -q " passed" "$OUT/pytest_gpu.log" && ! grep -q "failed" "$OUT/pytest_gpu.log" || { echo "GPU tests failed"; exit 1; }
TAG=${TAG:-r02d} bash tools/profile.sh || exit $?
