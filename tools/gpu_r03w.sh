#!/bin/bash
# r03w: rate dematcher at 8 waves/SIMD (64 VGPRs, 4 spilled): DL-SCH tests, A/B e2e + ue_dl (twice), e2e timeline
set -e
OUT=gpurun_out/r03w
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_dlsch_gpu.py tests/test_pdsch_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
bash tools/ab_uedl.sh srsran_amd/lib_var/prev.so srsran_amd/lib_var/new.so > $OUT/ab.txt 2>&1
bash tools/trace_pdsch.sh r03w
echo rc=0
