# usage: bash tools/gpu_r5t.sh: fused Adam + operand prep: A/B against separate launches
set -o pipefail
timeout -k 10 300 python -u tools/ab_fold.py > gpurun_out/r5t_ab.log 2>&1
rc=$?
grep -v "^frame\|Warn" gpurun_out/r5t_ab.log | tail -8; exit $rc
