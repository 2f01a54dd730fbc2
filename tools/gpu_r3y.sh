#!/bin/bash
# KLD: blocked T + slot-blocked compact gradient + staged merge (main) vs without the merge change (kbg), blocked T only (kbt), round-3 start (kold); bench KLD lines
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kld.py tests/test_gpu_kld_compact.py tests/test_gpu_optim.py > gpurun_out/r3y_tests.log 2>&1 || { tail -40 gpurun_out/r3y_tests.log; exit 1; }
tail -1 gpurun_out/r3y_tests.log
for P in 361 190; do
timeout -k 10 300 python3 tools/ab_libs.py --protos $P --call kldc --reps 30 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3y_ab_kldc$P.log
done
timeout -k 10 600 python -u bench.py --no-push --no-knn --no-eval --no-small-batch --no-train --no-sigmoid > gpurun_out/r3y_bench.log 2>&1 || { tail -30 gpurun_out/r3y_bench.log; exit 1; }
python3 - <<'PY'
import json
l=[x for x in open('gpurun_out/r3y_bench.log') if x.startswith('{')][-1]
d=json.loads(l); print(d['value'], d['ms_per_step']); print(json.dumps(d.get('kld_step')))
PY
