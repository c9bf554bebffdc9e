#!/bin/bash
# double-buffered DL-SCH descriptor scratch / softbuffer reset lists: DL-SCH / PDSCH / ue_dl / drop-in GPU tests, A/B
set -e
OUT=gpurun_out/r03db
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_dlsch_gpu.py tests/test_pdsch_gpu.py tests/test_pdcch_gpu.py tests/test_ue_dl_gpu.py tests/test_dropin_gpu.py tests/test_uedl_chunks_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
bash tools/ab_uedl.sh srsran_amd/lib_var/new.so srsran_amd/lib_var/dbuf.so > $OUT/ab.txt 2>&1
bash tools/trace_uedl.sh r03db > /dev/null 2>&1
echo rc=0
