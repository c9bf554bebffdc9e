set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_tdec_gpu.py tests/test_dlsch_gpu.py tests/test_srslte_tdec_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mapv_tests.log 2>&1 && bash tools/ab3.sh srsran_amd/lib/libsrsran_amd.so srsran_amd/lib_var/w3.so srsran_amd/lib_var/old.so > gpurun_out/mapv_ab.txt 2>&1
echo rc=$?
