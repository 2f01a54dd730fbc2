#!/bin/bash
set -u
mkdir -p gpurun_out
PROTOSEG_BWD=onepass timeout -k 10 300 python tools/ab_libs.py --protos 361 --call bwd_full --reps 30 > gpurun_out/abvar1.log 2>&1 || { tail -5 gpurun_out/abvar1.log; exit 1; }
grep -v amdgpu.ids gpurun_out/abvar1.log | tail -4
