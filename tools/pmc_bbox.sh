#!/bin/bash
# SQ / LDS / HBM counter passes over tools/bbox_time.py (upsample + bound boxes, 190 maps);
# one counter group per pass, kernel trace only.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-bbox}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o p$i --output-format csv -- \
    python3 "$R/tools/bbox_time.py" 2 > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"; tail -n 1 "$OUT/p$i.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 "$R/tools/pmc_summary.py" "$OUT" > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt"
