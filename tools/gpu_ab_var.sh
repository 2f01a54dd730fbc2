#!/bin/bash
# Interleaved A/B of the build_var/* libraries (one-pass backward) at P = 361 and 190.
set -u
mkdir -p gpurun_out
for P in 361 190; do
  PROTOSEG_BWD=onepass timeout -k 10 300 python tools/ab_libs.py --protos $P --call bwd_full --reps 30 > gpurun_out/abvar_$P.log 2>&1 || { tail -5 gpurun_out/abvar_$P.log; exit 1; }
  echo "== P=$P"; grep -v amdgpu.ids gpurun_out/abvar_$P.log | tail -6
done
