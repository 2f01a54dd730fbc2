#!/bin/bash
# spill-free fused backward, div_pix in the bf16 family, phase-B prefetch depth: parity + A/B
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_l2.py tests/test_gpu_kld_compact.py tests/test_gpu_kld.py tests/test_gpu_onepass.py > gpurun_out/r3u_tests.log 2>&1 || { tail -40 gpurun_out/r3u_tests.log; exit 1; }
tail -1 gpurun_out/r3u_tests.log
timeout -k 10 400 python3 tools/ab_libs.py --protos 361 --call bwd_full --reps 30 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3u_ab_bwd361.log
timeout -k 10 400 python3 tools/ab_libs.py --protos 190 --call bwd_full --reps 30 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3u_ab_bwd190.log
timeout -k 10 400 python3 tools/ab_libs.py --protos 361 --call fwd --reps 30 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3u_ab_fwd361.log
