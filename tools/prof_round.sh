#!/bin/bash
# Per-kernel profile of the prototype layer: ablation timings, phase stamps (stamps build) and
# SQ/LDS counters (tools/pmc_sq.sh), summarised into gpurun_out/pmc_summary.txt.
set -u
R=$(pwd)
mkdir -p gpurun_out
export TAG=${TAG:-s2}
timeout -k 10 200 python tools/ablate.py --reps 20 > gpurun_out/ablate.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ablate.log
L=$R/adlm-inherently-interpretable-segmentation_amd/csrc/build_stamps/libprotoseg_hip.so
PROTOSEG_HIP_LIB=$L timeout -k 10 120 python tools/stamps.py > gpurun_out/stamps_fwd.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/stamps_fwd.log
PROTOSEG_HIP_LIB=$L timeout -k 10 120 python tools/stamps_pw.py > gpurun_out/stamps_pw.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/stamps_pw.log
bash tools/pmc_sq.sh > gpurun_out/pmc_sq_run.log 2>&1 || exit $?
python tools/pmc_summary.py gpurun_out/pmc_$TAG > gpurun_out/pmc_summary.txt 2>&1
cat gpurun_out/pmc_summary.txt
