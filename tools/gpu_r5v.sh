# usage: bash tools/gpu_r5v.sh: slab-reduce groups per workgroup (4 / 8 / 16), interleaved backward A/B
set -o pipefail
timeout -k 10 300 python -u tools/ab_libs.py --protos 361 --call bwd_full --reps 40 > gpurun_out/r5v_361.log 2>&1 \
 && timeout -k 10 300 python -u tools/ab_libs.py --protos 361 --batch 2 --call bwd_full --reps 40 > gpurun_out/r5v_361b2.log 2>&1
rc=$?
tail -4 gpurun_out/r5v_361.log gpurun_out/r5v_361b2.log; exit $rc
