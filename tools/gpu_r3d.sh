#!/bin/bash
set -u
bash tools/gpu_ab_bwd.sh || exit $?
PROTOSEG_BWD=onepass TAG=one190b DRIVER_ARGS="--P 190" bash tools/pmc_bwd.sh > /dev/null 2>&1 || exit $?
PROTOSEG_BWD=onepass TAG=one361b DRIVER_ARGS="--P 361" bash tools/pmc_bwd.sh > /dev/null 2>&1 || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_one190b | tail -4
python3 tools/pmc_summary.py gpurun_out/pmc_one361b | tail -4
