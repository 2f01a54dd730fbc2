#!/bin/bash
# full GPU suite, one-pass stamps (P=361 / 190), bench defaults
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r3g_tests.log 2>&1 || { tail -30 gpurun_out/r3g_tests.log; exit 1; }
tail -3 gpurun_out/r3g_tests.log
CS=adlm-inherently-interpretable-segmentation_amd/csrc
for P in 361 190; do
  PROTOSEG_HIP_LIB=$CS/build_stamps/libprotoseg_hip.so PROTOSEG_BWD=onepass P=$P timeout -k 10 120 python -u tools/stamps_onepass.py > gpurun_out/r3g_stamps_$P.log 2>&1 || { tail -30 gpurun_out/r3g_stamps_$P.log; exit 1; }
  cat gpurun_out/r3g_stamps_$P.log | grep -v amdgpu.ids
done
timeout -k 10 500 python -u bench.py > gpurun_out/r3g_bench.log 2>&1 || { tail -30 gpurun_out/r3g_bench.log; exit 1; }
tail -c 1500 gpurun_out/r3g_bench.log
