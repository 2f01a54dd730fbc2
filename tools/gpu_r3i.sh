#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kld_compact.py tests/test_gpu_kld.py tests/test_gpu_l2.py > gpurun_out/r3i_tests.log 2>&1 || { tail -40 gpurun_out/r3i_tests.log; exit 1; }
tail -2 gpurun_out/r3i_tests.log
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for P in 190 361; do
P=$P timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r3i_prof_$P" -o kp --output-format csv -- python3 "$R/tools/kld_prof.py" > "$R/gpurun_out/r3i_prof_$P.log" 2>&1 || { tail -20 "$R/gpurun_out/r3i_prof_$P.log"; exit 1; }
cut -d, -f1-4 $(find "$R/gpurun_out/r3i_prof_$P" -name "*kernel_stats.csv") | head -16
done
cd "$R"
timeout -k 10 500 python -u bench.py --no-train --no-push --no-knn --no-eval --no-small-batch --no-cpu-baseline > gpurun_out/r3i_bench.log 2>&1 || { tail -30 gpurun_out/r3i_bench.log; exit 1; }
python3 - <<'PY'
import json
l=[x for x in open('gpurun_out/r3i_bench.log') if x.startswith('{')][-1]
d=json.loads(l); print(d['value'], d['ms_per_step']); print(json.dumps(d.get('kld_step')))
PY
