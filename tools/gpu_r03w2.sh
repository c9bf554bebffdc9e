#!/bin/bash
# sequential blind-search walk: control / ue_dl / drop-in / matrix GPU tests, kernel times and ue_dl A/B
set -e
OUT=gpurun_out/r03w2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_pdcch_gpu.py tests/test_ue_dl_gpu.py tests/test_dropin_gpu.py tests/test_uedl_chunks_gpu.py tests/test_phy_dl_matrix_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
bash tools/gpu_blindtrace.sh srsran_amd/lib_var/new.so srsran_amd/lib_var/walk.so > $OUT/bt.txt 2>&1
bash tools/ab_uedl.sh srsran_amd/lib_var/new.so srsran_amd/lib_var/walk.so > $OUT/ab.txt 2>&1
echo rc=0
