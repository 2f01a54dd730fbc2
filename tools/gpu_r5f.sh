# usage: TAG=r5f bash tools/gpu_r5f.sh: wide-family bf16x3 mode: GPU tests, configs[4] / reference-default timings per precision
set -o pipefail
t=${TAG:-r5f}
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_l2.py tests/test_gpu_push.py > gpurun_out/${t}_tests.log 2>&1 \
 && timeout -k 10 120 python -u tools/wide_run.py c4 10 bf16x3 > gpurun_out/${t}_c4.log 2>&1 \
 && timeout -k 10 120 python -u tools/wide_run.py c4 10 f32 > gpurun_out/${t}_c4_f32.log 2>&1 \
 && timeout -k 10 120 python -u tools/wide_run.py ref 10 bf16x3 > gpurun_out/${t}_ref.log 2>&1
rc=$?
tail -15 gpurun_out/${t}_tests.log; grep -h "ms_per_step" gpurun_out/${t}_c4*.log gpurun_out/${t}_ref.log | cut -c1-600; exit $rc
