#!/bin/bash
# A/B of the two training-backward kernels (PROTOSEG_BWD=fused | onepass) on the headline step.
set -u
mkdir -p gpurun_out
for k in fused onepass; do
  PROTOSEG_BWD=$k timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-push --no-kld --no-knn --no-eval > gpurun_out/ab_$k.log 2>&1 || { tail -5 gpurun_out/ab_$k.log; exit 1; }
  echo "== $k"; grep -v amdgpu.ids gpurun_out/ab_$k.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('P361 ms', d['ms_per_step'], d['kernels']); print('P190', d.get('protos_190',{}).get('ms_per_step'), d.get('protos_190',{}).get('kernels'))"
done
