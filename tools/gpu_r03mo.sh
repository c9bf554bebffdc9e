#!/bin/bash
# descrambling and conversion micro-optimisations in the LLR code: parity suites, kernel times
set -e
OUT=gpurun_out/r03mo
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_dlsch_gpu.py tests/test_configs_gpu.py tests/test_phy_dl_matrix_gpu.py tests/test_pdsch_gpu.py tests/test_ue_dl_gpu.py tests/test_dropin_gpu.py tests/test_uedl_chunks_gpu.py tests/test_eq_rm_gpu.py tests/test_real_signal.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
bash tools/gpu_eqk.sh srsran_amd/lib_var/lean.so srsran_amd/lib_var/mo.so srsran_amd/lib_var/lean.so srsran_amd/lib_var/mo.so > $OUT/ek.txt 2>&1
echo rc=0
