#!/bin/bash
# r03v: TB epilogue CRC24A with slice-by-4 tables and precomputed per-thread scale factors: DL-SCH / PDSCH / drop-in /
# config tests, A/B e2e + ue_dl, e2e timeline
set -e
OUT=gpurun_out/r03v
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_dlsch_gpu.py tests/test_dlsch8_gpu.py tests/test_pdsch_gpu.py tests/test_pdsch8_gpu.py tests/test_dropin_gpu.py tests/test_configs_gpu.py tests/test_ue_dl_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
bash tools/ab_uedl.sh srsran_amd/lib_var/prev.so srsran_amd/lib_var/new.so > $OUT/ab.txt 2>&1
bash tools/trace_pdsch.sh r03v
echo rc=0
