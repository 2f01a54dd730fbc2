# usage: bash tools/gpu_r5y.sh: push wave-kernel launch plan (chunk width / workgroups) vs the fixed plan; push tests
set -o pipefail
for a in "--images 8 --protos 190" "--images 1 --protos 190" "--images 8 --protos 361" "--images 1 --protos 361" "--images 2 --protos 190"; do
  echo "== $a" >> gpurun_out/r5y_ab.log
  timeout -k 10 300 python -u tools/ab_push.py $a --reps 30 >> gpurun_out/r5y_ab.log 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_push.py > gpurun_out/r5y_tests.log 2>&1
rc=$?
grep -v Warn gpurun_out/r5y_ab.log | grep -v amdgpu.ids; tail -2 gpurun_out/r5y_tests.log; exit $rc
