#!/bin/bash
# W per subcarrier in pdsch_eq_rm: parity suites, kernel times vs the previous build
set -e
OUT=gpurun_out/r03wc
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_dlsch_gpu.py tests/test_configs_gpu.py tests/test_phy_dl_matrix_gpu.py tests/test_pdsch_gpu.py tests/test_ue_dl_gpu.py tests/test_dropin_gpu.py tests/test_uedl_chunks_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
bash tools/gpu_eqk.sh srsran_amd/lib_var/lean.so srsran_amd/lib_var/wcol.so srsran_amd/lib_var/lean.so srsran_amd/lib_var/wcol.so > $OUT/ek.txt 2>&1
echo rc=0
