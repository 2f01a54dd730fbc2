# usage: bash tools/gpu_r5x.sh: KLD pixel-range length (1024 / 2048 / 4352 pixels per workgroup), interleaved A/B
set -o pipefail
for a in "--protos 361 --call kldc" "--protos 190 --call kldc" "--protos 361 --batch 4 --call kldc"; do
  timeout -k 10 300 python -u tools/ab_libs.py $a --reps 40 >> gpurun_out/r5x_ab.log 2>&1 || exit $?
done
grep -v Warn gpurun_out/r5x_ab.log | grep -v amdgpu.ids
