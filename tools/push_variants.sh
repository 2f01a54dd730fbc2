#!/bin/bash
# Variant libraries of push.hip only (-D knobs), linked with the main build's other objects:
#   tools/push_variants.sh NAME "-DKNOB=V ..." -> adlm-.../csrc/build_var/NAME/libprotoseg_hip.so
set -eu
NAME=$1; FLAGS=$2
CSRC=$(cd "$(dirname "$0")/../adlm-inherently-interpretable-segmentation_amd/csrc" && pwd)
OUT=$CSRC/build_var/$NAME
mkdir -p "$OUT"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function $FLAGS -I$CSRC/../../include -I$CSRC \
  -c $CSRC/push.hip -o $OUT/push.o
objs=""
for s in capi l2_layer l2_bf16 l2_bwd_fused kld eval knn bbox; do objs="$objs $CSRC/$s.o"; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC $objs $OUT/push.o -o $OUT/libprotoseg_hip.so
echo "built $OUT/libprotoseg_hip.so"
