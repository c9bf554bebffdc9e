#!/bin/bash
# r03u: blind decoder at 5,152 B of LDS per wave (31 waves / CU) + fused-check payload as dword stores: control,
# DL-SCH / PDSCH / config tests, A/B e2e + ue_dl, timelines
set -e
OUT=gpurun_out/r03u
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_dlsch_gpu.py tests/test_pdsch_gpu.py tests/test_configs_gpu.py tests/test_pdcch_gpu.py tests/test_real_signal.py tests/test_real_signal_10m.py tests/test_dropin_gpu.py tests/test_phy_dl_matrix_gpu.py tests/test_uedl_chunks_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
bash tools/ab_uedl.sh srsran_amd/lib_var/prev.so srsran_amd/lib_var/new.so > $OUT/ab.txt 2>&1
bash tools/trace_uedl.sh r03u
bash tools/trace_pdsch.sh r03t
echo rc=0
