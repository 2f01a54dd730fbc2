#!/bin/bash
# SQ/LDS counter passes over tools/ablate.py variants, or over CMD (a python3 argument list, e.g.
# CMD="tools/wide_run.py c4 5", relative to the repo root); one counter group per pass, kernel trace only — never combined
# with other tracing domains. TRAFFIC=1 adds a FETCH_SIZE and a WRITE_SIZE pass.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-sq}
ONLY=${ONLY:-fwd_dist_logits,bwd_x,bwd_pw}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES" \
           ${TRAFFIC:+"FETCH_SIZE" "WRITE_SIZE"}; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o p$i --output-format csv -- \
    python3 $R/${CMD:-tools/ablate.py --reps 3 --only "$ONLY" ${ABLATE_ARGS:-}} > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"; tail -n 2 "$OUT/p$i.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
