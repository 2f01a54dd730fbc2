#!/bin/bash
# build_var.sh NAME SRC.hip [extra hipcc flags...]: a variant library in csrc/build_var/NAME with
# l2_bwd_onepass.o compiled from SRC (and flags), every other object from the main build.
set -eu
C=$(cd "$(dirname "$0")/../adlm-inherently-interpretable-segmentation_amd/csrc" && pwd)
name=$1; src=$2; shift 2
d=$C/build_var/$name
mkdir -p "$d"
cp "$src" "$d/l2_bwd_onepass.hip"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function "$@" -I"$C/../../include" -I"$C" -c "$d/l2_bwd_onepass.hip" -o "$d/l2_bwd_onepass.o"
objs=""
for o in capi l2_layer l2_wide l2_bf16 l2_bwd_fused push kld eval knn bbox adam; do objs="$objs $C/$o.o"; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC $objs "$d/l2_bwd_onepass.o" -o "$d/libprotoseg_hip.so"
echo "built $d"
