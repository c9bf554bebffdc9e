set -o pipefail
bash tools/tdec_diag.sh > gpurun_out/diag_summary.txt 2>&1
echo rc=$?
