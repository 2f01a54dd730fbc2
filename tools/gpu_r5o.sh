# usage: bash tools/gpu_r5o.sh: wide-family tests + configs[4] / reference-default timings (128-tile bf16x3), then the full verification (tools/gpu_fin.sh)
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wide.py > gpurun_out/r5o_wtests.log 2>&1 \
 && timeout -k 10 120 python -u tools/wide_run.py c4 10 bf16x3 > gpurun_out/r5o_c4.log 2>&1 \
 && timeout -k 10 120 python -u tools/wide_run.py ref 10 bf16x3 > gpurun_out/r5o_ref.log 2>&1
rc=$?
tail -3 gpurun_out/r5o_wtests.log; grep -h ms_per_step gpurun_out/r5o_c4.log gpurun_out/r5o_ref.log | cut -c1-700
[ $rc -eq 0 ] || exit $rc
TAG=r5fa bash tools/gpu_fin.sh
