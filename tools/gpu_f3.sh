set -u
mkdir -p gpurun_out/f9
timeout -k 10 300 python -u -m pytest tests/test_gpu_l2.py tests/test_gpu_kld.py -x -q --timeout 120 --timeout-method thread > gpurun_out/f9/l2.log 2>&1
rc=$?; tail -5 gpurun_out/f9/l2.log
if [ $rc -ne 0 ]; then tail -60 gpurun_out/f9/l2.log; exit $rc; fi
timeout -k 10 120 python tools/ablate.py --reps 20 --only bwd_full,bwd_x,bwd_pw > gpurun_out/f9/ab190.log 2>&1 || exit $?
timeout -k 10 120 python tools/ablate.py --reps 20 --protos 361 --only bwd_full > gpurun_out/f9/ab361.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/f9/ab190.log gpurun_out/f9/ab361.log
L=$(pwd)/adlm-inherently-interpretable-segmentation_amd/csrc/build_stamps/libprotoseg_hip.so
PROTOSEG_HIP_LIB=$L timeout -k 10 120 python tools/stamps_fused.py > gpurun_out/f9/st190.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/f9/st190.log
