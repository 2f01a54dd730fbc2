#!/bin/bash
# A/B kernel timings: tools/ablate.py against the main library and each build_var/* variant,
# plus the forward stamps of the stamps build.
set -u
mkdir -p gpurun_out
C=adlm-inherently-interpretable-segmentation_amd/csrc
echo "== main"; timeout -k 10 120 python tools/ablate.py --reps 30 2>&1 | grep -v amdgpu.ids || exit $?
for d in $C/build_var/*/; do
  n=$(basename $d); echo "== $n"
  PROTOSEG_HIP_LIB=$d/libprotoseg_hip.so timeout -k 10 120 python tools/ablate.py --reps 30 2>&1 | grep -v amdgpu.ids || exit $?
done
if [ -f $C/build_stamps/libprotoseg_hip.so ]; then
  echo "== stamps fwd"; PROTOSEG_HIP_LIB=$C/build_stamps/libprotoseg_hip.so timeout -k 10 120 python tools/stamps.py 2>&1 | grep -v amdgpu.ids || exit $?
fi
