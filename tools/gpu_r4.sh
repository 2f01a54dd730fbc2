#!/bin/bash
# Round-4 GPU runner: gpu_r4.sh <step>...  (run on the GPU box from the repo root; each step has
# its own time limit and the script stops at the first failure).
#   tests   full -m gpu suite          smoke   __graft_entry__.smoke()
#   bench   default bench.py line      prof    rocprofv3 kernel stats of the P=361 / P=190 steps
#   sq      SQ counters of the one-pass backward
set -u
mkdir -p gpurun_out
T=${TAG:-r4}
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
        > gpurun_out/${T}_tests.log 2>&1 || { tail -60 gpurun_out/${T}_tests.log; exit 1; }
      tail -3 gpurun_out/${T}_tests.log ;;
    tests-new)
      timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
        tests/test_gpu_headline_parity.py tests/test_gpu_kld_compact.py tests/test_checkpoint.py tests/test_gpu_dp_capture.py \
        > gpurun_out/${T}_tests_new.log 2>&1 || { tail -60 gpurun_out/${T}_tests_new.log; exit 1; }
      tail -30 gpurun_out/${T}_tests_new.log ;;
    ptest)  # PT_FILES="tests/a.py tests/b.py"
      timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${PT_FILES} \
        > gpurun_out/${T}_ptest.log 2>&1 || { tail -60 gpurun_out/${T}_ptest.log; exit 1; }
      tail -3 gpurun_out/${T}_ptest.log ;;
    quick-noops)
      PROTOSEG_FWD_OPERANDS=0 timeout -k 10 300 python -u bench.py --no-kld --no-push --no-knn --no-eval --no-train --no-sigmoid --no-cpu-baseline --no-wide \
        > gpurun_out/${T}_quick_noops.log 2>&1 || { tail -30 gpurun_out/${T}_quick_noops.log; exit 1; }
      python3 tools/bench_summary.py gpurun_out/${T}_quick_noops.log ;;
    diag)
      timeout -k 10 300 python -u tools/debug/kld_compact_diag.py > gpurun_out/${T}_diag.log 2>&1; tail -30 gpurun_out/${T}_diag.log ;;
    smoke)
      timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/${T}_smoke.log 2>&1 \
        || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
      tail -1 gpurun_out/${T}_smoke.log ;;
    bench)
      timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 || { tail -30 gpurun_out/${T}_bench.log; exit 1; }
      python3 tools/bench_summary.py gpurun_out/${T}_bench.log ;;
    quick)
      timeout -k 10 300 python -u bench.py --no-kld --no-push --no-knn --no-eval --no-train --no-sigmoid --no-cpu-baseline --no-wide \
        > gpurun_out/${T}_quick.log 2>&1 || { tail -30 gpurun_out/${T}_quick.log; exit 1; }
      python3 tools/bench_summary.py gpurun_out/${T}_quick.log ;;
    wide)
      timeout -k 10 300 python -u bench.py --no-kld --no-push --no-knn --no-eval --no-train --no-sigmoid --no-cpu-baseline --no-small-batch --side-protos 0 --steps 10 \
        > gpurun_out/${T}_wide.log 2>&1 || { tail -30 gpurun_out/${T}_wide.log; exit 1; }
      python3 tools/bench_summary.py gpurun_out/${T}_wide.log ;;
    prof)
      TAG=$T WORKLOADS="p361 p190" bash tools/profile.sh > gpurun_out/${T}_profile.log 2>&1 \
        || { tail -20 gpurun_out/${T}_profile.log; exit 1; }
      for wl in p361 p190; do python3 tools/kstats.py gpurun_out/prof_$T/$wl/trace/trace_kernel_stats.csv; done ;;
    sq)
      TAG=onepass361_$T DRIVER_ARGS="--P 361" bash tools/pmc_bwd.sh > gpurun_out/${T}_pmc.log 2>&1 \
        || { tail -20 gpurun_out/${T}_pmc.log; exit 1; }
      tail -25 gpurun_out/${T}_pmc.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
