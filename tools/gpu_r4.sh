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
    widetrace)  # rocprofv3 kernel trace of each wide configuration alone (per-launch table)
      for cfg in c4 ref; do
        ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/wt_${T}_$cfg" \
            -o wt --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/wide_run.py" $cfg 10 \
            > "$GRAFT_REPO_ROOT/gpurun_out/${T}_wt_$cfg.log" 2>&1 ) || { tail -20 gpurun_out/${T}_wt_$cfg.log; exit 1; }
        tail -1 gpurun_out/${T}_wt_$cfg.log
        python3 tools/ktrace_grid.py $(find gpurun_out/wt_${T}_$cfg -name '*kernel_trace.csv')
      done ;;
    steptrace)  # kernel trace of the KLD step and the small-batch layer steps, each alone
      for spec in "kld --protos 361" "kld --protos 190" "layer --protos 361 --batch 2" "layer --protos 361 --batch 4" "layer --protos 361"; do
        tag=$(echo "$spec" | tr -d ' -' )
        ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/st_${T}_$tag" \
            -o st --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/step_trace.py" $spec \
            > "$GRAFT_REPO_ROOT/gpurun_out/${T}_st_$tag.log" 2>&1 ) || { tail -20 gpurun_out/${T}_st_$tag.log; exit 1; }
        grep "ms/step" gpurun_out/${T}_st_$tag.log
        python3 tools/ktrace_grid.py $(find gpurun_out/st_${T}_$tag -name '*kernel_trace.csv')
      done ;;
    abkld)  # interleaved A/B of the build_var/* KLD variants against the main build
      for P in 361 190; do
        for c in kld kldc; do
          timeout -k 10 300 python -u tools/ab_libs.py --protos $P --call $c --reps 40 > gpurun_out/${T}_ab_${c}_$P.log 2>&1 \
            || { tail -20 gpurun_out/${T}_ab_${c}_$P.log; exit 1; }
          tail -6 gpurun_out/${T}_ab_${c}_$P.log
        done
      done ;;
    abbwdk)  # interleaved A/B of the build_var/* variants on the layer backward with the compact KLD gradient
      for P in 361 190; do
        timeout -k 10 300 python -u tools/ab_libs.py --protos $P --call bwdk --reps 40 > gpurun_out/${T}_ab_bwdk_$P.log 2>&1 \
          || { tail -20 gpurun_out/${T}_ab_bwdk_$P.log; exit 1; }
        tail -4 gpurun_out/${T}_ab_bwdk_$P.log
      done ;;
    abbwd)  # interleaved A/B of the build_var/* variants on the plain layer backward
      for P in 361 190; do
        timeout -k 10 300 python -u tools/ab_libs.py --protos $P --call bwd_full --reps 40 > gpurun_out/${T}_ab_bwd_$P.log 2>&1 \
          || { tail -20 gpurun_out/${T}_ab_bwd_$P.log; exit 1; }
        tail -6 gpurun_out/${T}_ab_bwd_$P.log
      done ;;
    abmask)  # interleaved A/B of the build_var/* variants on the patch class mask (8 Cityscapes labels)
      timeout -k 10 300 python -u tools/ab_libs.py --protos 190 --call mask --reps 40 > gpurun_out/${T}_ab_mask.log 2>&1 \
        || { tail -20 gpurun_out/${T}_ab_mask.log; exit 1; }
      tail -4 gpurun_out/${T}_ab_mask.log ;;
    abfwdsb)  # interleaved A/B of the build_var/* variants on the small-batch forward
      for B in 2 4 8; do
        timeout -k 10 300 python -u tools/ab_libs.py --protos 361 --batch $B --call fwd --reps 40 > gpurun_out/${T}_ab_fwd_B$B.log 2>&1 \
          || { tail -20 gpurun_out/${T}_ab_fwd_B$B.log; exit 1; }
        tail -3 gpurun_out/${T}_ab_fwd_B$B.log
      done ;;
    stampskld)  # per-wave phase stamps of the KLD partial kernel (make stamps build)
      for P in 361 190; do
        PROTOSEG_HIP_LIB=$PWD/adlm-inherently-interpretable-segmentation_amd/csrc/build_stamps/libprotoseg_hip.so \
          timeout -k 10 300 python -u tools/stamps_kld.py $P > gpurun_out/${T}_stamps_kld_$P.log 2>&1 \
          || { tail -20 gpurun_out/${T}_stamps_kld_$P.log; exit 1; }
        grep -v "^W20" gpurun_out/${T}_stamps_kld_$P.log | tail -10
      done ;;
    evalb)  # the bench's eval line alone (plus the headline step it always runs)
      timeout -k 10 300 python -u bench.py --no-kld --no-push --no-knn --no-train --no-sigmoid --no-cpu-baseline --no-wide \
        --no-small-batch --side-protos 0 > gpurun_out/${T}_evalb.log 2>&1 || { tail -30 gpurun_out/${T}_evalb.log; exit 1; }
      python3 tools/bench_summary.py gpurun_out/${T}_evalb.log ;;
    abchunk)  # interleaved A/B of the build_var/* variants at P = 570 (two prototype chunks)
      for c in fwd bwd_full; do
        timeout -k 10 300 python -u tools/ab_libs.py --protos 570 --call $c --reps 30 > gpurun_out/${T}_ab_${c}_570.log 2>&1 \
          || { tail -20 gpurun_out/${T}_ab_${c}_570.log; exit 1; }
        tail -3 gpurun_out/${T}_ab_${c}_570.log
      done ;;
    abpush)  # interleaved A/B of the build_var/* push variants on the argmin call (8 maps)
      for P in 190 361; do
        timeout -k 10 300 python -u tools/ab_libs.py --protos $P --call push --reps 40 > gpurun_out/${T}_ab_push_$P.log 2>&1 \
          || { tail -20 gpurun_out/${T}_ab_push_$P.log; exit 1; }
        tail -4 gpurun_out/${T}_ab_push_$P.log
      done ;;
    pushtrace)  # kernel trace of the push inner step alone
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/pt_${T}" \
          -o pt --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/push_trace.py" 8 20 \
          > "$GRAFT_REPO_ROOT/gpurun_out/${T}_pt.log" 2>&1 ) || { tail -20 gpurun_out/${T}_pt.log; exit 1; }
      tail -1 gpurun_out/${T}_pt.log
      python3 tools/ktrace_grid.py $(find gpurun_out/pt_${T} -name '*kernel_trace.csv') ;;
    abfwd)  # interleaved A/B of the build_var/* variants on the forward call
      for P in 361 190; do
        timeout -k 10 300 python -u tools/ab_libs.py --protos $P --call fwd --reps 40 > gpurun_out/${T}_ab_fwd_$P.log 2>&1 \
          || { tail -20 gpurun_out/${T}_ab_fwd_$P.log; exit 1; }
        tail -4 gpurun_out/${T}_ab_fwd_$P.log
      done ;;
    sqwide)  # SQ counters over the configs[4] wide step alone
      TAG=wide_c4_$T DRIVER=tools/wide_run.py DRIVER_ARGS="c4 3" bash tools/pmc_bwd.sh > gpurun_out/${T}_sqwide.log 2>&1 \
        || { tail -20 gpurun_out/${T}_sqwide.log; exit 1; }
      grep -E "wide_gemm|derived" gpurun_out/${T}_sqwide.log | head -20 ;;
    sqpush)  # SQ counters over the push inner step alone
      TAG=push_$T DRIVER=tools/push_trace.py DRIVER_ARGS="8 5" bash tools/pmc_bwd.sh > gpurun_out/${T}_sqpush.log 2>&1 \
        || { tail -20 gpurun_out/${T}_sqpush.log; exit 1; }
      grep -E "push_argmin|patch_mask|derived" gpurun_out/${T}_sqpush.log | head -20 ;;
    profall)  # the three profile workloads (trace + FETCH_SIZE + WRITE_SIZE passes each)
      TAG=$T WORKLOADS="p361 p190 rest" bash tools/profile.sh > gpurun_out/${T}_profile.log 2>&1 \
        || { tail -20 gpurun_out/${T}_profile.log; exit 1; }
      for wl in p361 p190 rest; do python3 tools/kstats.py gpurun_out/prof_$T/$wl/trace/trace_kernel_stats.csv; done ;;
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
