#!/bin/bash
# forward distance-store cache policy: plain (main) vs nt (cp2), sc1 (cp16), sc0 sc1 (cp17)
set -u
mkdir -p gpurun_out
for P in 361 190; do
timeout -k 10 300 python3 tools/ab_libs.py --protos $P --call fwd --reps 40 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3aa_ab_fwd$P.log
done
