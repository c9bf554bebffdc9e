#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/c4
timeout -k 10 400 python -u -m pytest tests/test_dlsch_gpu.py tests/test_dlsch8_gpu.py tests/test_pdsch_gpu.py tests/test_ue_dl_gpu.py tests/test_dropin_gpu.py tests/test_pdcch_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c4/test.log 2>&1 && \
bash tools/ab_kstats.sh srsran_amd/lib_var/head.so srsran_amd/lib/libsrsran_amd.so dlsch_cb_check
echo rc=$?
