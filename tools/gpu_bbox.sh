#!/bin/bash
# Bound-box kernels: parity tests, the standalone timing, then a kernel-trace pass of the timing.
set -u
OUT=${OUT:-gpurun_out/bbox}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_bbox.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -n 3 "$OUT/tests.log"; if [ $rc -ne 0 ]; then tail -n 40 "$OUT/tests.log"; exit $rc; fi
timeout -k 10 200 python tools/bbox_time.py 10 > "$OUT/time.log" 2>&1 || { tail -n 30 "$OUT/time.log"; exit 1; }
grep -v amdgpu.ids "$OUT/time.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $GRAFT_REPO_ROOT/$OUT/prof -o b --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bbox_time.py 5 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || exit $?
cat $(find $GRAFT_REPO_ROOT/$OUT/prof -name "*kernel_stats.csv")
