#!/bin/bash
# build_var.sh NAME SRC.hip [extra hipcc flags...]: a variant library in csrc/build_var/NAME with
# $OBJ.o (default l2_bwd_wave) compiled from SRC (and flags), every other object from the main build.
set -eu
C=$(cd "$(dirname "$0")/../adlm-inherently-interpretable-segmentation_amd/csrc" && pwd)
name=$1; src=$2; shift 2
obj=${OBJ:-l2_bwd_wave}
# the Makefile's per-object flags
extra=""
[ "$obj" = bbox ] && extra="-ffp-contract=off"
d=$C/build_var/$name
mkdir -p "$d"
cp "$src" "$d/$obj.hip"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $extra "$@" -I"$C/../../include" -I"$C" -c "$d/$obj.hip" -o "$d/$obj.o"
objs=""
for o in capi l2_layer l2_wide l2_bf16 l2_bwd_fused l2_bwd_wave push kld eval knn bbox adam; do
  [ "$o" = "$obj" ] || objs="$objs $C/$o.o"
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC $objs "$d/$obj.o" -o "$d/libprotoseg_hip.so"
echo "built $d"
