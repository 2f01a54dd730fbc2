#!/bin/bash
# Interleaved A/B of build_var/* against the main library (tools/ab_libs.py) + the l2 GPU tests.
set -u
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_l2.py tests/test_gpu_kld.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/l2_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/ab/l2_tests.log; if [ $rc -ne 0 ]; then tail -n 40 gpurun_out/ab/l2_tests.log; exit $rc; fi
for spec in ${AB_SPECS:-"bwd_full 361" "bwd_full 190" "bwd_full_xsig 361" "fwd 361"}; do
  set -- $spec
  timeout -k 10 180 python tools/ab_libs.py --call $1 --protos $2 --reps ${REPS:-40} 2>&1 | grep -v amdgpu.ids || exit $?
done
