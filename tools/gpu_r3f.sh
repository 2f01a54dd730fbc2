#!/bin/bash
# one-pass parity + optimizer tests, then the bench with the new side lines
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_onepass.py tests/test_gpu_l2.py tests/test_gpu_optim.py > gpurun_out/r3f_tests.log 2>&1 || { tail -30 gpurun_out/r3f_tests.log; exit 1; }
tail -3 gpurun_out/r3f_tests.log
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3f_bench.log 2>&1 || { tail -30 gpurun_out/r3f_bench.log; exit 1; }
tail -c 3000 gpurun_out/r3f_bench.log
