# usage: bash tools/gpu_ab.sh TAG [ab_libs args...]: interleaved A/B of the build_var libraries
set -o pipefail
tag=$1; shift
timeout -k 10 300 python -u tools/ab_libs.py "$@" > gpurun_out/ab_$tag.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/ab_$tag.log | tail -12; exit $rc
