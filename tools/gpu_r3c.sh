#!/bin/bash
set -u
PROTOSEG_BWD=onepass TAG=one190 DRIVER_ARGS="--P 190" bash tools/pmc_bwd.sh || exit $?
PROTOSEG_BWD=fused TAG=fus190 DRIVER_ARGS="--P 190" bash tools/pmc_bwd.sh || exit $?
