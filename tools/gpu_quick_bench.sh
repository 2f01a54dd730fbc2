#!/bin/bash
# Quick loop: named GPU tests, then the P = 361 / 190 layer-step bench lines and a kernel-trace pass.
set -u
mkdir -p gpurun_out/qb
timeout -k 10 300 python -u -m pytest ${QB_TESTS:-tests/test_gpu_optim.py} -x -q --timeout 120 --timeout-method thread > gpurun_out/qb/tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/qb/tests.log; if [ $rc -ne 0 ]; then tail -n 40 gpurun_out/qb/tests.log; exit $rc; fi
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-push --no-knn --no-eval > gpurun_out/qb/bench.log 2>&1 || { tail -n 30 gpurun_out/qb/bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/qb/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('P361 ms', d['ms_per_step'], 'img/s', d['value'], d['kernels']); print('P190 ms', d['protos_190']['ms_per_step']); print('kld', d.get('kld_step', {}).get('ms_per_step'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $GRAFT_REPO_ROOT/gpurun_out/qb/prof -o q --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --protos 361 --side-protos 0 --no-kld --no-push --no-knn --no-eval > $GRAFT_REPO_ROOT/gpurun_out/qb/prof.log 2>&1 || exit $?
cat $(find $GRAFT_REPO_ROOT/gpurun_out/qb/prof -name "*kernel_stats.csv")
