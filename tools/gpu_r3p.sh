#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/ab_libs.py --protos 361 --call fwd --reps 40 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3p_ab_fwd361.log
timeout -k 10 300 python3 tools/ab_libs.py --protos 190 --call fwd --reps 40 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3p_ab_fwd190.log
