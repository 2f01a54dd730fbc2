#!/bin/bash
# Forward store-path / sigmoid-fusion ablations (P = 361 / 190, 65x65 vs 64x64 maps) and the
# P = 361 / 190 rocprofv3 passes (kernel stats + FETCH / WRITE) for the traffic table.
set -u
mkdir -p gpurun_out/r2s6
A="fwd_dist_logits,fwd_logits_only,fwd_dist_only,fwd_xsig,bwd_full,bwd_full_xsig"
for P in 361 190; do
  for F in 65 64; do
    echo "== P=$P fmap=$F"
    timeout -k 10 120 python tools/ablate.py --reps 30 --protos $P --fmap $F --only $A 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
TAG=r02c WORKLOADS="p361 p190" bash tools/profile.sh || exit $?
bash tools/ab_fused.sh || exit $?
