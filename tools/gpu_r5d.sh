# usage: TAG=r5d bash tools/gpu_r5d.sh: forward variant A/B, rocprofv3 of the p361 / p190 steps, default bench
set -o pipefail
t=${TAG:-r5d}
R=$(pwd)
timeout -k 10 200 python -u tools/ab_libs.py --protos 361 --call fwd --reps 40 > gpurun_out/${t}_abfwd361.log 2>&1 \
 && timeout -k 10 200 python -u tools/ab_libs.py --protos 190 --call fwd --reps 40 > gpurun_out/${t}_abfwd190.log 2>&1 \
 && TAG=$t WORKLOADS="p361 p190" bash tools/profile.sh > gpurun_out/${t}_prof.log 2>&1 \
 && cd "$R" && timeout -k 10 600 python -u bench.py > gpurun_out/${t}_bench.log 2>&1
rc=$?
cd "$R"; grep -hv amdgpu.ids gpurun_out/${t}_abfwd*.log; tail -c 3000 gpurun_out/${t}_bench.log; exit $rc
