#!/bin/bash
# Kernel ablations at several batch sizes / map sides: separates the transcendental cost, the
# per-launch fixed cost (startup + tail) and the distance-store cost (aligned vs unaligned rows).
set -u
mkdir -p gpurun_out/abl
for cfg in "32 65" "32 64" "128 65" "128 64"; do
  set -- $cfg
  echo "== batch $1 fmap $2"
  timeout -k 10 200 python tools/ablate.py --reps 20 --batch $1 --fmap $2 --only fwd_dist_logits,fwd_dist_only,fwd_logits_only > gpurun_out/abl/b$1_f$2.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/abl/b$1_f$2.log
done
