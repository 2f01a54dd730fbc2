#!/bin/bash
# compact KLD gradient: new parity tests, KLD + l2 suites, then the bench
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kld_compact.py tests/test_gpu_kld.py > gpurun_out/r3h_tests.log 2>&1 || { tail -40 gpurun_out/r3h_tests.log; exit 1; }
tail -3 gpurun_out/r3h_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r3h_all.log 2>&1 || { tail -40 gpurun_out/r3h_all.log; exit 1; }
tail -3 gpurun_out/r3h_all.log
timeout -k 10 500 python -u bench.py --no-train > gpurun_out/r3h_bench.log 2>&1 || { tail -30 gpurun_out/r3h_bench.log; exit 1; }
python3 - <<'PY'
import json
l=[x for x in open('gpurun_out/r3h_bench.log') if x.startswith('{')][-1]
d=json.loads(l); print(d['value'], d['ms_per_step']); print(json.dumps(d.get('kld_step'), indent=1))
PY
