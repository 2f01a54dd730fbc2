#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_wide.py > gpurun_out/r3j_wide.log 2>&1 || { tail -60 gpurun_out/r3j_wide.log; exit 1; }
grep -E "passed|failed" gpurun_out/r3j_wide.log | tail -2
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r3j_all.log 2>&1 || { tail -40 gpurun_out/r3j_all.log; exit 1; }
tail -2 gpurun_out/r3j_all.log
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for P in 190 361; do
P=$P timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r3j_prof_$P" -o kp --output-format csv -- python3 "$R/tools/kld_prof.py" > "$R/gpurun_out/r3j_prof_$P.log" 2>&1 || { tail -20 "$R/gpurun_out/r3j_prof_$P.log"; exit 1; }
cut -d, -f1-4 $(find "$R/gpurun_out/r3j_prof_$P" -name "*kernel_stats.csv") | head -16
done
