#!/bin/bash
# Short GPU loop: gpu tests for the layer, kernel ablation timings, one bench line.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_l2.py tests/test_gpu_kld.py -x -q --timeout 120 --timeout-method thread > gpurun_out/q_tests.log 2>&1
rc=$?; tail -3 gpurun_out/q_tests.log; if [ $rc -ne 0 ]; then tail -40 gpurun_out/q_tests.log; exit $rc; fi
timeout -k 10 200 python tools/ablate.py --reps 20 > gpurun_out/q_ablate.log 2>&1 || exit $?
cat gpurun_out/q_ablate.log | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-push > gpurun_out/q_bench.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/q_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms/step', d['ms_per_step'], d['kernels'])"
