#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/ab_libs.py --protos 190 --call push --reps 30 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3n_ab_push190.log
timeout -k 10 300 python3 tools/ab_libs.py --protos 361 --call push --reps 30 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3n_ab_push361.log
