# usage: bash tools/gpu_r5z.sh: push wave kernel with 4-wave workgroups (2 per CU) vs 8; push / operands tests; fold A/B (1024-thread adam_prep)
set -o pipefail
for a in "--images 8 --protos 190" "--images 1 --protos 190" "--images 8 --protos 361" "--images 1 --protos 361"; do
  echo "== $a" >> gpurun_out/r5z_ab.log
  timeout -k 10 300 python -u tools/ab_push.py $a --reps 30 >> gpurun_out/r5z_ab.log 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_push.py tests/test_gpu_operands.py > gpurun_out/r5z_tests.log 2>&1 \
 && timeout -k 10 300 python -u tools/ab_fold.py 32,361 2,361 > gpurun_out/r5z_fold.log 2>&1
rc=$?
grep -v Warn gpurun_out/r5z_ab.log | grep -v amdgpu.ids | grep -v "vs block"; tail -2 gpurun_out/r5z_tests.log; grep "B=" gpurun_out/r5z_fold.log; exit $rc
