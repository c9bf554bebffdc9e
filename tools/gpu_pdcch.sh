#!/bin/bash
# control-channel changes: their GPU tests, then the find_and_decode trace
set -o pipefail
mkdir -p gpurun_out/pd
timeout -k 10 400 python -u -m pytest tests/test_pdcch_gpu.py tests/test_real_signal.py tests/test_real_signal_10m.py tests/test_dropin_gpu.py tests/test_ue_dl_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pd/test.log 2>&1 && \
bash tools/trace_uedl.sh pd
echo rc=$?
