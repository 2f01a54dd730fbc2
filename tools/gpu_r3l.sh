#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kld_compact.py tests/test_gpu_kld.py > gpurun_out/r3l_tests.log 2>&1 || { tail -40 gpurun_out/r3l_tests.log; exit 1; }
tail -2 gpurun_out/r3l_tests.log
timeout -k 10 300 python3 tools/ab_libs.py --protos 361 --call fwd --reps 40 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3l_ab_fwd361.log
timeout -k 10 300 python3 tools/ab_libs.py --protos 190 --call fwd --reps 40 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3l_ab_fwd190.log
timeout -k 10 300 python3 tools/ab_libs.py --protos 361 --call bwd_full --reps 40 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3l_ab_bwd361.log
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for P in 190 361; do
P=$P timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r3l_prof_$P" -o kp --output-format csv -- python3 "$R/tools/kld_prof.py" > "$R/gpurun_out/r3l_prof_$P.log" 2>&1 || { tail -20 "$R/gpurun_out/r3l_prof_$P.log"; exit 1; }
python3 "$R/tools/kstats.py" "$R/gpurun_out/r3l_prof_$P/kp_kernel_stats.csv" | grep kld
done
