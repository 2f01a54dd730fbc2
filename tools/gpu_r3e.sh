#!/bin/bash
set -u
C=adlm-inherently-interpretable-segmentation_amd/csrc
PROTOSEG_BWD=onepass PROTOSEG_HIP_LIB=$C/build_stamps/libprotoseg_hip.so P=361 timeout -k 10 120 python tools/stamps_onepass.py 2>&1 | grep -v amdgpu.ids
PROTOSEG_BWD=onepass PROTOSEG_HIP_LIB=$C/build_stamps/libprotoseg_hip.so P=190 timeout -k 10 120 python tools/stamps_onepass.py 2>&1 | grep -v amdgpu.ids
