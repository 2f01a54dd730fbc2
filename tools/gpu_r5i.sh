# usage: TAG=r5i bash tools/gpu_r5i.sh: wave-streamed push argmin: GPU push tests + A/B vs the block kernel
set -o pipefail
t=${TAG:-r5i}
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_push.py tests/test_gpu_bbox.py tests/test_gpu_knn.py > gpurun_out/${t}_tests.log 2>&1 \
 && timeout -k 10 200 python -u tools/ab_push.py --images 8 --protos 190 > gpurun_out/${t}_ab8.log 2>&1 \
 && timeout -k 10 200 python -u tools/ab_push.py --images 1 --protos 190 > gpurun_out/${t}_ab1.log 2>&1 \
 && timeout -k 10 200 python -u tools/ab_push.py --images 8 --protos 361 > gpurun_out/${t}_ab8_361.log 2>&1
rc=$?
tail -5 gpurun_out/${t}_tests.log; grep -hv amdgpu.ids gpurun_out/${t}_ab*.log; exit $rc
