#!/bin/bash
# blind decoder: lane-major decision strings + lane-walking traceback, rotating (default) and identity (v0) layouts
set -e
OUT=gpurun_out/r03v3
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_pdcch_gpu.py tests/test_ue_dl_gpu.py tests/test_dropin_gpu.py tests/test_uedl_chunks_gpu.py tests/test_phy_dl_matrix_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
MI355_LIB=srsran_amd/lib_var/v0.so timeout -k 10 300 python -u -m pytest tests/test_pdcch_gpu.py tests/test_ue_dl_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests_v0.log 2>&1
bash tools/gpu_blindtrace.sh srsran_amd/lib_var/prev.so srsran_amd/lib_var/v0.so srsran_amd/lib_var/new.so > $OUT/bt.txt 2>&1
echo rc=0
