#!/bin/bash
# Round 3, first GPU pass: the push-tie / optimizer tests, then the headline bench without
# side lines (a fresh baseline for the fused-backward work).
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_push.py tests/test_gpu_optim.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3a_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r3a_tests.log; if [ $rc -ne 0 ]; then tail -60 gpurun_out/r3a_tests.log; exit $rc; fi
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-push > gpurun_out/r3a_bench.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r3a_bench.log | tail -1 | head -c 1500
