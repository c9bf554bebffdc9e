#!/bin/bash
# blind decoder in the rotating state layout: blind-search / ue_dl / drop-in GPU tests, then A/B vs the previous build
set -e
OUT=gpurun_out/r03v2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_pdcch_gpu.py tests/test_ue_dl_gpu.py tests/test_dropin_gpu.py tests/test_uedl_chunks_gpu.py tests/test_phy_dl_matrix_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
bash tools/ab_uedl.sh srsran_amd/lib_var/prev.so srsran_amd/lib_var/new.so > $OUT/ab.txt 2>&1
echo rc=0
