#!/bin/bash
# one-pass backward knobs, all built with the product's max-ilp scheduler unless named: main vs
# s_setprio for waves 4-7 (prio), no per-k-step fence in phase B (pbfree), default scheduler
# (defsched), prefetch depth 1 (pb1); then phase stamps of the stamped build
set -u
mkdir -p gpurun_out
timeout -k 10 400 python3 tools/ab_libs.py --protos 361 --call bwd_full --reps 40 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3ab_ab_bwd361.log
CS=$(pwd)/adlm-inherently-interpretable-segmentation_amd/csrc
PROTOSEG_HIP_LIB=$CS/build_stamps/libprotoseg_hip.so PROTOSEG_BWD=onepass P=361 timeout -k 10 120 python -u tools/stamps_onepass.py > gpurun_out/r3ab_stamps_361.log 2>&1 || { tail -30 gpurun_out/r3ab_stamps_361.log; exit 1; }
tail -25 gpurun_out/r3ab_stamps_361.log
