# usage: bash tools/gpu_fwdabl.sh TAG: forward ablation A/B (build_var variants) at P = 361 / 190 and the store probe
set -o pipefail
t=$1
timeout -k 10 200 python -u tools/ab_libs.py --protos 361 --call fwd --reps 40 > gpurun_out/${t}_fwd361.log 2>&1 \
 && timeout -k 10 200 python -u tools/ab_libs.py --protos 361 --fmap 64 --call fwd --reps 40 > gpurun_out/${t}_fwd361_64.log 2>&1 \
 && timeout -k 10 60 ./tools/probe/store_bw.bin 4225 361 > gpurun_out/${t}_store4225.log 2>&1 \
 && timeout -k 10 60 ./tools/probe/store_bw.bin 4224 361 > gpurun_out/${t}_store4224.log 2>&1
rc=$?
grep -hv amdgpu.ids gpurun_out/${t}_*.log; exit $rc
