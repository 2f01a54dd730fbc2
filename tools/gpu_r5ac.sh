# usage: bash tools/gpu_r5ac.sh: 16-B slab reduce vs the scalar one (interleaved backward A/B), headline parity / operands tests
set -o pipefail
for a in "--protos 361 --call bwd_full" "--protos 361 --batch 2 --call bwd_full" "--protos 570 --call bwd_full"; do
  timeout -k 10 300 python -u tools/ab_libs.py $a --reps 40 >> gpurun_out/r5ac_ab.log 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_headline_parity.py tests/test_gpu_operands.py tests/test_gpu_l2.py > gpurun_out/r5ac_tests.log 2>&1
rc=$?
grep -v Warn gpurun_out/r5ac_ab.log | grep -v amdgpu.ids; tail -2 gpurun_out/r5ac_tests.log; exit $rc
