# usage: bash tools/gpu_r5q.sh: kernel trace of the configs[4] wide step (fp16 X, bf16x3)
set -o pipefail
R=$(pwd); mkdir -p gpurun_out/prof_r5q
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -T -d "$R/gpurun_out/prof_r5q" -o c4 --output-format csv -- python3 "$R/tools/wide_run.py" c4 10 bf16x3 > "$R/gpurun_out/prof_r5q/c4.log" 2>&1
rc=$?
cd "$R"; python3 tools/kstats.py gpurun_out/prof_r5q/c4_kernel_stats.csv 2>/dev/null | head -30 || head -30 gpurun_out/prof_r5q/c4_kernel_stats.csv; exit $rc
