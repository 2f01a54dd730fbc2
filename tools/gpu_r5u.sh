# usage: bash tools/gpu_r5u.sh: step-by-step folded layer step (eager, then graph replays)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/dbg_fold.py 32 361 separate > gpurun_out/r5u_sep.log 2>&1 \
 && timeout -k 10 120 python -u tools/dbg_fold.py 32 361 fold > gpurun_out/r5u_fold.log 2>&1
rc=$?
grep -v "^frame\|Warn" gpurun_out/r5u_sep.log | tail -5; grep -v "^frame\|Warn" gpurun_out/r5u_fold.log | head -30; exit $rc
