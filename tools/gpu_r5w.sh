# usage: bash tools/gpu_r5w.sh: XCD-aware tile mapping (forward, wave / fused backward) vs the plain order
set -o pipefail
for a in "--protos 361 --call fwd" "--protos 361 --call bwd_full" "--protos 190 --call fwd" "--protos 190 --call bwd_full" "--protos 361 --batch 2 --call bwd_full"; do
  timeout -k 10 300 python -u tools/ab_libs.py $a --reps 40 >> gpurun_out/r5w_ab.log 2>&1 || exit $?
done
grep -v Warn gpurun_out/r5w_ab.log | grep -v amdgpu.ids
