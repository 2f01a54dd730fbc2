#!/bin/bash
# Round-3 final: full GPU suite, smoke(), per-config profiles + PMC traffic, SQ counters of the
# one-pass backward, KLD kernel stats, the default bench line.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r3fin_all.log 2>&1 || { tail -40 gpurun_out/r3fin_all.log; exit 1; }
tail -1 gpurun_out/r3fin_all.log
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > gpurun_out/r3fin_smoke.log 2>&1 || { tail -20 gpurun_out/r3fin_smoke.log; exit 1; }
tail -1 gpurun_out/r3fin_smoke.log
TAG=r03 WORKLOADS="p361 p190" bash tools/profile.sh > gpurun_out/r3fin_profile.log 2>&1 || { tail -20 gpurun_out/r3fin_profile.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_r03 gpurun_out/prof_r03.json --traffic > gpurun_out/r3fin_profsum.log 2>&1 || { tail -20 gpurun_out/r3fin_profsum.log; exit 1; }
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
TAG=onepass361_r3fin DRIVER_ARGS="--P 361" bash tools/pmc_bwd.sh > gpurun_out/r3fin_pmc.log 2>&1 || { tail -20 gpurun_out/r3fin_pmc.log; exit 1; }
tail -25 gpurun_out/r3fin_pmc.log
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for P in 190 361; do
P=$P timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r3fin_kld_$P" -o kp --output-format csv -- python3 "$R/tools/kld_prof.py" > "$R/gpurun_out/r3fin_kld_$P.log" 2>&1 || { tail -20 "$R/gpurun_out/r3fin_kld_$P.log"; exit 1; }
python3 "$R/tools/kstats.py" "$R/gpurun_out/r3fin_kld_$P/kp_kernel_stats.csv" | grep kld
done
cd "$R"
timeout -k 10 600 python -u bench.py > gpurun_out/r3fin_bench.log 2>&1 || { tail -30 gpurun_out/r3fin_bench.log; exit 1; }
python3 - <<'PY'
import json
l=[x for x in open('gpurun_out/r3fin_bench.log') if x.startswith('{')][-1]
d=json.loads(l); print(d['value'], d['ms_per_step'], d['kernels'], d['roofline']); print(json.dumps(d.get('kld_step'))); print(d['protos_190']['ms_per_step'])
PY
