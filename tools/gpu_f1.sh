set -u
mkdir -p gpurun_out/f1
timeout -k 10 300 python -u -m pytest tests/test_gpu_l2.py -x -q --timeout 120 --timeout-method thread > gpurun_out/f1/l2.log 2>&1
rc=$?; tail -30 gpurun_out/f1/l2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python tools/ablate.py --reps 20 --only bwd_full,bwd_x,bwd_pw,fwd_dist_logits > gpurun_out/f1/ab190.log 2>&1 || exit $?
timeout -k 10 120 python tools/ablate.py --reps 20 --protos 361 --only bwd_full,bwd_x,bwd_pw,fwd_dist_logits > gpurun_out/f1/ab361.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/f1/ab190.log gpurun_out/f1/ab361.log
