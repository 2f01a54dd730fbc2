#!/bin/bash
# forward phase stamps at the drop-in's small batches and at the bench batch (P = 361)
set -u
mkdir -p gpurun_out
CS=$(pwd)/adlm-inherently-interpretable-segmentation_amd/csrc
for B in 2 4 32; do
PROTOSEG_HIP_LIB=$CS/build_stamps/libprotoseg_hip.so B=$B P=361 timeout -k 10 120 python -u tools/stamps.py > gpurun_out/r3ae_fwd_stamps_B$B.log 2>&1 || { tail -30 gpurun_out/r3ae_fwd_stamps_B$B.log; exit 1; }
echo "== B=$B"; tail -14 gpurun_out/r3ae_fwd_stamps_B$B.log
done
