#!/bin/bash
# One-pass backward: GPU parity tests, then an A/B timing of the two backward kernels.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_onepass.py tests/test_gpu_optim.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3b_tests.log 2>&1
rc=$?; tail -25 gpurun_out/r3b_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
for k in fused onepass; do
  PROTOSEG_BWD=$k timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-push --no-kld --no-knn --no-eval > gpurun_out/r3b_bench_$k.log 2>&1 || exit $?
  echo "== $k"; grep -v amdgpu.ids gpurun_out/r3b_bench_$k.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('P361 ms', d['ms_per_step'], d['kernels']); print('P190', d.get('protos_190',{}).get('ms_per_step'), d.get('protos_190',{}).get('kernels'))"
done
