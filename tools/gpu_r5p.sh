# usage: bash tools/gpu_r5p.sh: wave backward with 2p sum g_s folded into its slab (reduce mode 2): parity tests, A/B vs build_var/old, configs[4] timing
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_onepass.py tests/test_gpu_kld_compact.py tests/test_gpu_operands.py tests/test_gpu_headline_parity.py tests/test_gpu_optim.py > gpurun_out/r5p_tests.log 2>&1 \
 && timeout -k 10 200 python -u tools/ab_libs.py --protos 361 --main-bwd wave --call bwd_full --reps 40 > gpurun_out/r5p_ab361.log 2>&1 \
 && timeout -k 10 120 python -u tools/wide_run.py c4 10 bf16x3 > gpurun_out/r5p_c4.log 2>&1
rc=$?
tail -3 gpurun_out/r5p_tests.log; grep -hv amdgpu.ids gpurun_out/r5p_ab361.log; grep -h ms_per_step gpurun_out/r5p_c4.log | cut -c1-400; exit $rc
