#!/bin/bash
# KLD forward as bucket + per-(class, image) group kernels; compact gradient per group: parity, then the bench's KLD lines under rocprof
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kld.py tests/test_gpu_kld_compact.py tests/test_gpu_optim.py > gpurun_out/r3w_tests.log 2>&1 || { tail -40 gpurun_out/r3w_tests.log; exit 1; }
tail -1 gpurun_out/r3w_tests.log
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for P in 190 361; do
P=$P timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r3w_prof_$P" -o kp --output-format csv -- python3 "$R/tools/kld_prof.py" > "$R/gpurun_out/r3w_prof_$P.log" 2>&1 || { tail -20 "$R/gpurun_out/r3w_prof_$P.log"; exit 1; }
python3 "$R/tools/kstats.py" "$R/gpurun_out/r3w_prof_$P/kp_kernel_stats.csv" | grep kld
done
cd "$R"
timeout -k 10 600 python -u bench.py --no-push --no-knn --no-eval --no-small-batch --no-train --no-sigmoid > gpurun_out/r3w_bench.log 2>&1 || { tail -30 gpurun_out/r3w_bench.log; exit 1; }
python3 - <<'PY'
import json
l=[x for x in open('gpurun_out/r3w_bench.log') if x.startswith('{')][-1]
d=json.loads(l); print(d['value'], d['ms_per_step']); print(json.dumps(d.get('kld_step')))
PY
