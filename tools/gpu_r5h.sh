# usage: TAG=r5h bash tools/gpu_r5h.sh: wave backward (fused reduce/convert, half-split g_dist loads) tests + A/B vs build_var/sep
set -o pipefail
t=${TAG:-r5h}
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_onepass.py tests/test_gpu_kld_compact.py tests/test_gpu_operands.py tests/test_gpu_headline_parity.py > gpurun_out/${t}_tests.log 2>&1 \
 && timeout -k 10 200 python -u tools/ab_libs.py --protos 361 --main-bwd wave --call bwd_full --reps 40 > gpurun_out/${t}_ab361.log 2>&1 \
 && timeout -k 10 200 python -u tools/ab_libs.py --protos 361 --main-bwd wave --call bwdk --reps 40 > gpurun_out/${t}_abk361.log 2>&1
rc=$?
tail -3 gpurun_out/${t}_tests.log; grep -hv amdgpu.ids gpurun_out/${t}_ab*.log; exit $rc
