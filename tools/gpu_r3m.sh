#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r3m_all.log 2>&1 || { tail -40 gpurun_out/r3m_all.log; exit 1; }
tail -2 gpurun_out/r3m_all.log
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for P in 190 361; do
P=$P timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r3m_prof_$P" -o kp --output-format csv -- python3 "$R/tools/kld_prof.py" > "$R/gpurun_out/r3m_prof_$P.log" 2>&1 || { tail -20 "$R/gpurun_out/r3m_prof_$P.log"; exit 1; }
python3 "$R/tools/kstats.py" "$R/gpurun_out/r3m_prof_$P/kp_kernel_stats.csv" | grep kld
done
cd "$R"
timeout -k 10 600 python -u bench.py > gpurun_out/r3m_bench.log 2>&1 || { tail -30 gpurun_out/r3m_bench.log; exit 1; }
python3 - <<'PY'
import json
l=[x for x in open('gpurun_out/r3m_bench.log') if x.startswith('{')][-1]
d=json.loads(l); print(d['value'], d['ms_per_step'], d['kernels']); print(json.dumps(d.get('kld_step'))); print(d['protos_190']['ms_per_step'], d['protos_190']['kernels'])
PY
