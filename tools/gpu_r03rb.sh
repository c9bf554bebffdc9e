#!/bin/bash
# DL-SCH pending read-back on its own stream: ue_dl / drop-in / chunk tests, A/B (pdsch, ue_dl) x 3 vs the previous build
set -e
OUT=gpurun_out/r03rb
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ue_dl_gpu.py tests/test_dropin_gpu.py tests/test_uedl_chunks_gpu.py tests/test_pdcch_gpu.py tests/test_eq_rm_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
bash tools/ab_uedl.sh srsran_amd/lib_var/lean.so srsran_amd/lib_var/rbq.so > $OUT/ab1.txt 2>&1
bash tools/ab_uedl.sh srsran_amd/lib_var/lean.so srsran_amd/lib_var/rbq.so > $OUT/ab2.txt 2>&1
echo rc=0
