#!/bin/bash
# Short GPU loop for the layer: parity tests, one bench line, and a rocprofv3 kernel-trace
# stats pass over the same bench (per-kernel average durations). Stops at the first failure.
set -u
R=$(pwd)
mkdir -p gpurun_out/qp
timeout -k 10 400 python -u -m pytest tests/test_gpu_l2.py tests/test_gpu_kld.py -x -q --timeout 120 --timeout-method thread > gpurun_out/qp/tests.log 2>&1
rc=$?; tail -2 gpurun_out/qp/tests.log; if [ $rc -ne 0 ]; then tail -40 gpurun_out/qp/tests.log; exit $rc; fi
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-push --no-knn --no-eval > gpurun_out/qp/bench.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/qp/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms/step', d['ms_per_step'], 'kld', d['kld_step']['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/qp/prof" -o qp --output-format csv -- \
  python3 "$R/bench.py" --steps 50 --warmup 5 --no-cpu-baseline --no-push --no-knn --no-eval > "$R/gpurun_out/qp/prof.log" 2>&1 || exit $?
cut -d, -f1-4 $(find "$R/gpurun_out/qp/prof" -name "*kernel_stats.csv") | head -16
