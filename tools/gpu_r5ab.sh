# usage: bash tools/gpu_r5ab.sh: wave backward under other machine schedulers (max-ilp / max-memory-clause / iterative-ilp), interleaved A/B
set -o pipefail
for a in "--protos 361 --call bwd_full" "--protos 361 --batch 2 --call bwd_full"; do
  timeout -k 10 300 python -u tools/ab_libs.py $a --reps 40 >> gpurun_out/r5ab_ab.log 2>&1 || exit $?
done
grep -v Warn gpurun_out/r5ab_ab.log | grep -v amdgpu.ids
