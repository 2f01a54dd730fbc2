#!/bin/bash
# round-3 profiles: push block A/B, kernel-trace + FETCH/WRITE passes per bench workload, SQ
# counters of the one-pass backward at P = 361
set -u
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/ab_libs.py --protos 190 --call push --reps 30 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3o_ab_push190.log
TAG=r03 WORKLOADS="p361 p190" bash tools/profile.sh || exit $?
python3 tools/prof_summary.py gpurun_out/prof_r03 gpurun_out/prof_r03.json --traffic || exit $?
TAG=onepass361 DRIVER_ARGS="--P 361" bash tools/pmc_bwd.sh > gpurun_out/pmc_onepass361.log 2>&1 || { tail -20 gpurun_out/pmc_onepass361.log; exit 1; }
tail -30 gpurun_out/pmc_onepass361.log
