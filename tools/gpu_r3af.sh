#!/bin/bash
# small-batch forward grid (main: remainder path up to 3 rounds) vs the previous grid (prev)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_l2.py tests/test_gpu_onepass.py tests/test_gpu_kld_compact.py > gpurun_out/r3af_tests.log 2>&1 || { tail -40 gpurun_out/r3af_tests.log; exit 1; }
tail -1 gpurun_out/r3af_tests.log
for B in 2 6 8 12 16 32; do
timeout -k 10 300 python3 tools/ab_libs.py --batch $B --protos 361 --call fwd --reps 40 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3af_ab_fwd_B$B.log
done
timeout -k 10 300 python3 tools/ab_libs.py --batch 4 --protos 190 --call fwd --reps 40 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3af_ab_fwd_B4_P190.log
