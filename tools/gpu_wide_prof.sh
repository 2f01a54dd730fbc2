#!/bin/bash
# usage: TAG=x bash tools/gpu_wide_prof.sh: rocprofv3 kernel stats of the two wide-family step
# configurations alone (tools/wide_run.py c4 / ref), into gpurun_out/prof_wide_$TAG/.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_wide_${TAG:-x}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for c in c4 ref; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/$c" -o "$c" --output-format csv -- python3 "$R/tools/wide_run.py" "$c" 10 \
    > "$OUT/$c.log" 2>&1 || exit $?
  tail -n 1 "$OUT/$c.log"
done
