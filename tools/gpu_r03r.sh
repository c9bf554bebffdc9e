#!/bin/bash
# r03r: blind decoder CRC16 / payload packing across lanes (no serial lane-0 loop): control tests, A/B ue_dl, SQ PMC
set -e
OUT=gpurun_out/r03r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_pdcch_gpu.py tests/test_real_signal.py tests/test_real_signal_10m.py tests/test_dropin_gpu.py tests/test_phy_dl_matrix_gpu.py tests/test_uedl_chunks_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
bash tools/ab_uedl.sh srsran_amd/lib_var/prev.so srsran_amd/lib_var/new.so > $OUT/ab.txt 2>&1
bash tools/pdcch_pmc.sh > $OUT/pmc.log 2>&1
echo rc=0
