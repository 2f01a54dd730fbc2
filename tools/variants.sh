#!/bin/bash
# Build in-tree variant libraries of the bf16 kernels (-D knobs) for A/B timing on the box:
#   tools/variants.sh NAME "-DKNOB=V ..."  ->  adlm-.../csrc/build_var/NAME/libprotoseg_hip.so
set -eu
NAME=$1; FLAGS=$2
CSRC=$(dirname "$0")/../adlm-inherently-interpretable-segmentation_amd/csrc
OUT=$CSRC/build_var/$NAME
mkdir -p "$OUT"
for s in capi l2_layer l2_bf16 l2_bwd_fused push kld eval knn bbox adam; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function $FLAGS -I$CSRC/../../include -I$CSRC -c $CSRC/$s.hip -o $OUT/$s.o &
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC $OUT/*.o -o $OUT/libprotoseg_hip.so
echo "built $OUT/libprotoseg_hip.so"
