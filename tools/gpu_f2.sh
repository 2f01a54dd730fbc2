set -u
mkdir -p gpurun_out/f2
L=$(pwd)/adlm-inherently-interpretable-segmentation_amd/csrc/build_stamps/libprotoseg_hip.so
PROTOSEG_HIP_LIB=$L timeout -k 10 120 python tools/stamps_fused.py > gpurun_out/f2/st190.log 2>&1 || exit $?
PROTOSEG_HIP_LIB=$L P=361 timeout -k 10 120 python tools/stamps_fused.py > gpurun_out/f2/st361.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/f2/st190.log gpurun_out/f2/st361.log
