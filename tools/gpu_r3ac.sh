#!/bin/bash
# one-pass phase stamps by wave index
set -u
mkdir -p gpurun_out
CS=$(pwd)/adlm-inherently-interpretable-segmentation_amd/csrc
PROTOSEG_HIP_LIB=$CS/build_stamps/libprotoseg_hip.so PROTOSEG_BWD=onepass P=361 timeout -k 10 120 python -u tools/stamps_onepass.py > gpurun_out/r3ac_stamps_361.log 2>&1 || { tail -30 gpurun_out/r3ac_stamps_361.log; exit 1; }
tail -12 gpurun_out/r3ac_stamps_361.log
