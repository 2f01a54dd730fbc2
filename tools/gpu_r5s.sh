# usage: bash tools/gpu_r5s.sh: kernel-trace timelines of the KLD and plain steps (P = 361, B = 32 and 2)
set -o pipefail
R=$(pwd); mkdir -p gpurun_out/r5s; cd /tmp && export TMPDIR=/tmp
for cfg in "kld 32" "layer 32" "kld 2" "layer 2"; do
  set -- $cfg
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r5s/$1_$2 -o t -- python3 $R/tools/step_trace.py $1 --protos 361 --batch $2 --steps 10 > $R/gpurun_out/r5s/$1_$2.log 2>&1 || exit $?
  tail -1 $R/gpurun_out/r5s/$1_$2.log
done
