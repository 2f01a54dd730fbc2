# usage: bash tools/gpu_r5z2.sh: operands / optimizer tests (adam_update without contraction), fold A/B (1024-thread adam_prep)
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_operands.py tests/test_gpu_optim.py > gpurun_out/r5z2_tests.log 2>&1 \
 && timeout -k 10 300 python -u tools/ab_fold.py 32,361 2,361 > gpurun_out/r5z2_fold.log 2>&1
rc=$?
tail -2 gpurun_out/r5z2_tests.log; grep "B=" gpurun_out/r5z2_fold.log; exit $rc
