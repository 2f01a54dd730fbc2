# usage: TAG=r5g bash tools/gpu_r5g.sh: slab-reduce group A/B (build_var rg8 / rg16 vs main, wave backward) and push block A/B (blk8)
set -o pipefail
t=${TAG:-r5g}
timeout -k 10 200 python -u tools/ab_libs.py --protos 361 --main-bwd wave --call bwd_full --reps 40 > gpurun_out/${t}_abred361.log 2>&1 \
 && timeout -k 10 200 python -u tools/ab_libs.py --protos 190 --call bwd_full --reps 40 > gpurun_out/${t}_abred190.log 2>&1 \
 && timeout -k 10 200 python -u tools/ab_libs.py --protos 190 --call push --reps 30 > gpurun_out/${t}_abpush.log 2>&1
rc=$?
grep -hv amdgpu.ids gpurun_out/${t}_ab*.log; exit $rc
