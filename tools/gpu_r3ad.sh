#!/bin/bash
# KLD chunk sizes: main (partial 256, gradient 128) vs gradient 256 (g256), partial 128 (p128), gradient 64 (g64)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kld.py tests/test_gpu_kld_compact.py > gpurun_out/r3ad_tests.log 2>&1 || { tail -40 gpurun_out/r3ad_tests.log; exit 1; }
tail -1 gpurun_out/r3ad_tests.log
for P in 361 190; do
timeout -k 10 300 python3 tools/ab_libs.py --protos $P --call kldc --reps 30 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3ad_ab_kldc$P.log
done
