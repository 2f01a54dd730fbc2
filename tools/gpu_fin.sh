# usage: TAG=r5fin bash tools/gpu_fin.sh: the full GPU suite, smoke, default bench, rocprofv3 passes (p361 / p190 / rest)
set -o pipefail
t=${TAG:-r5fin}
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${t}_gputests.log 2>&1 \
 && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > gpurun_out/${t}_smoke.log 2>&1 \
 && timeout -k 10 900 python -u bench.py > gpurun_out/${t}_bench.log 2>&1 \
 && TAG=$t WORKLOADS="${WL:-p361 p190 rest}" bash tools/profile.sh > gpurun_out/${t}_prof.log 2>&1
rc=$?
cd "$R"; tail -3 gpurun_out/${t}_gputests.log; tail -1 gpurun_out/${t}_smoke.log; tail -c 1500 gpurun_out/${t}_bench.log; tail -4 gpurun_out/${t}_prof.log; exit $rc
