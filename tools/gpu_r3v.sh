#!/bin/bash
# Round-3 checkpoint: full GPU suite, smoke(), clean per-config profiles (trace + PMC traffic), bench.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r3v_all.log 2>&1 || { tail -40 gpurun_out/r3v_all.log; exit 1; }
tail -2 gpurun_out/r3v_all.log
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > gpurun_out/r3v_smoke.log 2>&1 || { tail -20 gpurun_out/r3v_smoke.log; exit 1; }
tail -1 gpurun_out/r3v_smoke.log
TAG=r03 WORKLOADS="p361 p190" bash tools/profile.sh || exit 1
python3 tools/prof_summary.py gpurun_out/prof_r03 gpurun_out/prof_r03.json --traffic > gpurun_out/r3v_profsum.log 2>&1 || { tail -20 gpurun_out/r3v_profsum.log; exit 1; }
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
timeout -k 10 600 python -u bench.py > gpurun_out/r3v_bench.log 2>&1 || { tail -30 gpurun_out/r3v_bench.log; exit 1; }
python3 - <<'PY'
import json
l=[x for x in open('gpurun_out/r3v_bench.log') if x.startswith('{')][-1]
d=json.loads(l); print(d['value'], d['ms_per_step'], d['kernels'], d['roofline']); print(json.dumps(d.get('kld_step'))); print(d['protos_190']['ms_per_step'], d['protos_190']['kernels'])
PY
