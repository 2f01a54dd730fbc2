set -u
R=$(pwd)
mkdir -p gpurun_out
export TAG=s2
timeout -k 10 200 python tools/ablate.py --reps 20 > gpurun_out/ablate.log 2>&1; echo "ablate rc=$?"; cat gpurun_out/ablate.log | tail -6
PROTOSEG_HIP_LIB=$R/adlm-inherently-interpretable-segmentation_amd/csrc/build_stamps/libprotoseg_hip.so timeout -k 10 120 python tools/stamps.py > gpurun_out/stamps_fwd.log 2>&1; echo "stamps rc=$?"; cat gpurun_out/stamps_fwd.log
PROTOSEG_HIP_LIB=$R/adlm-inherently-interpretable-segmentation_amd/csrc/build_stamps/libprotoseg_hip.so timeout -k 10 120 python tools/stamps_pw.py > gpurun_out/stamps_pw.log 2>&1; echo "stamps_pw rc=$?"; cat gpurun_out/stamps_pw.log
bash tools/pmc_sq.sh > gpurun_out/pmc_sq_run.log 2>&1; echo "pmc rc=$?"; tail -5 gpurun_out/pmc_sq_run.log
python tools/pmc_summary.py gpurun_out/pmc_s2 > gpurun_out/pmc_summary.txt 2>&1; cat gpurun_out/pmc_summary.txt
