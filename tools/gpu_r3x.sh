#!/bin/bash
# KLD: register-blocked T and per-pixel gradient columns (main) vs previous (kold), fast divisions only (kfd), + blocked T (kbt)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kld.py tests/test_gpu_kld_compact.py > gpurun_out/r3x_tests.log 2>&1 || { tail -40 gpurun_out/r3x_tests.log; exit 1; }
tail -1 gpurun_out/r3x_tests.log
for P in 361 190; do
timeout -k 10 300 python3 tools/ab_libs.py --protos $P --call kld --reps 30 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3x_ab_kld$P.log
timeout -k 10 300 python3 tools/ab_libs.py --protos $P --call kldc --reps 30 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3x_ab_kldc$P.log
done
