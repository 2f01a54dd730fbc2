#!/bin/bash
# A/B of the fused backward: tools/ablate.py bwd_full against the main library and each
# build_var/* variant (P = 190 and 361).
set -u
C=adlm-inherently-interpretable-segmentation_amd/csrc
for P in 190 361; do
  echo "== main P=$P"; timeout -k 10 120 python tools/ablate.py --reps 30 --protos $P --only bwd_full 2>&1 | grep -v amdgpu.ids || exit $?
  for d in $C/build_var/*/; do
    n=$(basename $d); echo "== $n P=$P"
    PROTOSEG_HIP_LIB=$d/libprotoseg_hip.so timeout -k 10 120 python tools/ablate.py --reps 30 --protos $P --only bwd_full 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
