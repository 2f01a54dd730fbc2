# usage: TAG=x bash tools/gpu_r5a.sh: the wave backward's GPU tests and its A/B against onepass / fused
set -o pipefail
t=${TAG:-r5a}
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_onepass.py -k "wave" > gpurun_out/${t}_tests.log 2>&1 \
 && timeout -k 10 200 python -u tools/ab_bwd.py --protos 361 --kernels onepass,wave --reps 30 > gpurun_out/${t}_ab361.log 2>&1 \
 && timeout -k 10 200 python -u tools/ab_bwd.py --protos 190 --kernels fused,wave --reps 30 > gpurun_out/${t}_ab190.log 2>&1 \
 && timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kld_compact.py tests/test_gpu_operands.py > gpurun_out/${t}_tests2.log 2>&1
rc=$?
tail -3 gpurun_out/${t}_tests.log; grep -hv amdgpu.ids gpurun_out/${t}_ab*.log; tail -3 gpurun_out/${t}_tests2.log
exit $rc
