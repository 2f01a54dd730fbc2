# usage: bash tools/gpu_r5n.sh: SQ counters of the wave push kernel and the wave backward (P = 361)
set -o pipefail
TAG=r5push bash tools/pmc_push.sh > gpurun_out/pmc_r5push.log 2>&1 \
 && TAG=r5wave DRIVER_ARGS="--protos 361" bash tools/pmc_bwd.sh > gpurun_out/pmc_r5wave.log 2>&1
rc=$?
tail -25 gpurun_out/pmc_r5push.log; tail -25 gpurun_out/pmc_r5wave.log; exit $rc
