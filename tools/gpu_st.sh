set -u
mkdir -p gpurun_out/$1
L=$(pwd)/adlm-inherently-interpretable-segmentation_amd/csrc/build_stamps/libprotoseg_hip.so
PROTOSEG_HIP_LIB=$L timeout -k 10 120 python tools/stamps_fused.py > gpurun_out/$1/st190.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/$1/st190.log
