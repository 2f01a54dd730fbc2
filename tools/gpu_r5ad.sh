# usage: bash tools/gpu_r5ad.sh: KLD partial / compact-gradient kernels at 4 / 6 waves per EU vs 5 (interleaved A/B)
set -o pipefail
for a in "--protos 361 --call kldc" "--protos 190 --call kldc" "--protos 361 --batch 4 --call kldc"; do
  timeout -k 10 300 python -u tools/ab_libs.py $a --reps 40 >> gpurun_out/r5ad_ab.log 2>&1 || exit $?
done
grep -v Warn gpurun_out/r5ad_ab.log | grep -v amdgpu.ids
