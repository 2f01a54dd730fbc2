# usage: TAG=r5e bash tools/gpu_r5e.sh: wide-family tests (fp16 native), configs[4] fp16 vs f32 timing, KLD-backward kernel A/B
set -o pipefail
t=${TAG:-r5e}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wide.py tests/test_capi.py > gpurun_out/${t}_tests.log 2>&1 \
 && timeout -k 10 120 python -u tools/wide_run.py c4 > gpurun_out/${t}_c4.log 2>&1 \
 && timeout -k 10 120 python -u tools/wide_run.py c4f32 > gpurun_out/${t}_c4f32.log 2>&1 \
 && timeout -k 10 200 python -u tools/ab_libs.py --protos 361 --main-bwd wave,onepass --call bwdk --reps 30 > gpurun_out/${t}_abk361.log 2>&1 \
 && timeout -k 10 200 python -u tools/ab_libs.py --protos 190 --main-bwd wave,fused --call bwdk --reps 30 > gpurun_out/${t}_abk190.log 2>&1
rc=$?
tail -3 gpurun_out/${t}_tests.log; grep -h "ms_per_step" gpurun_out/${t}_c4*.log | cut -c1-400; grep -hv amdgpu.ids gpurun_out/${t}_abk*.log; exit $rc
