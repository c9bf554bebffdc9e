#!/bin/bash
# r03il: interleaved two-layer image in pdsch_eq_rm -- eq_rm parity tests, A/B against the per-layer images
# (srsran_amd/lib_var/il0.so, built with -DPDSCH_ER_IL=0), per-dispatch kernel trace
set -e
OUT=gpurun_out/r03il
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_eq_rm_gpu.py tests/test_configs_gpu.py tests/test_phy_dl_matrix_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
bash tools/gpu_eqk.sh srsran_amd/lib/libsrsran_amd.so srsran_amd/lib_var/il0.so srsran_amd/lib/libsrsran_amd.so srsran_amd/lib_var/il0.so > $OUT/ab.txt 2>&1
bash tools/gpu_ktrace.sh il
echo rc=0
