# usage: bash tools/gpu_r5ae.sh: push tests + rocprofv3 stats of the push line (8 and 1 images per call) with the batched merge loads
set -o pipefail
R=$(pwd)
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_push.py tests/test_gpu_bbox.py > gpurun_out/r5ae_tests.log 2>&1 || { tail -3 gpurun_out/r5ae_tests.log; exit 1; }
tail -1 gpurun_out/r5ae_tests.log
cd /tmp && export TMPDIR=/tmp
for n in 8 1; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5ae_$n -o s --output-format csv -- python3 $R/tools/push_trace.py $n 20 > $R/gpurun_out/r5ae_$n.log 2>&1 || exit $?
  grep -E "push_|patch_mask" $R/gpurun_out/r5ae_$n/s_kernel_stats.csv | cut -d, -f1-4
done
