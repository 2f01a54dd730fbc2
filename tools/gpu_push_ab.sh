#!/bin/bash
# push argmin A/B over the main build and build_var/* (tools/push_ab.py), then the GPU push tests.
set -u
C=adlm-inherently-interpretable-segmentation_amd/csrc
for L in $C/libprotoseg_hip.so $C/build_var/*/libprotoseg_hip.so; do
  PROTOSEG_HIP_LIB=$L timeout -k 10 100 python tools/push_ab.py 2>&1 | grep -v amdgpu.ids || exit $?
done
