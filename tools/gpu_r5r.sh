# usage: bash tools/gpu_r5r.sh: wide backward from saved distances: wide / l2 / checkpoint tests, configs[4] and reference-default timings
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_l2.py tests/test_gpu_operands.py > gpurun_out/r5r_tests.log 2>&1 \
 && timeout -k 10 120 python -u tools/wide_run.py c4 10 bf16x3 > gpurun_out/r5r_c4.log 2>&1 \
 && timeout -k 10 120 python -u tools/wide_run.py ref 10 bf16x3 > gpurun_out/r5r_ref.log 2>&1
rc=$?
tail -3 gpurun_out/r5r_tests.log; grep -h ms_per_step gpurun_out/r5r_c4.log gpurun_out/r5r_ref.log | cut -c1-500; exit $rc
