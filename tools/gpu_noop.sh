#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/no
timeout -k 10 400 python -u -m pytest tests/test_tdec_gpu.py tests/test_srslte_tdec_gpu.py tests/test_dlsch_gpu.py tests/test_dlsch8_gpu.py tests/test_pdsch_gpu.py tests/test_dropin_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/no/test.log 2>&1 && \
bash tools/ab_lib.sh srsran_amd/lib_var/r02g.so srsran_amd/lib/libsrsran_amd.so && bash tools/ab_lib.sh srsran_amd/lib_var/r02g.so srsran_amd/lib/libsrsran_amd.so
echo rc=$?
