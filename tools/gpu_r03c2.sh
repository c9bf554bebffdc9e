#!/bin/bash
# r03c2: estimator pilot gathers issued up front, MAP no-op launches exit before any other load -- parity, A/B
# (srsran_amd/lib_var/chest0.so)
set -e
OUT=gpurun_out/r03c2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tdec_gpu.py tests/test_dlsch_gpu.py tests/test_chest_state_gpu.py tests/test_ue_dl_gpu.py tests/test_wiener_gpu.py tests/test_channel_gpu.py tests/test_dropin_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
KF=chest_estimate,tdec_win_halfit bash tools/gpu_eqk.sh srsran_amd/lib/libsrsran_amd.so srsran_amd/lib_var/chest0.so srsran_amd/lib/libsrsran_amd.so srsran_amd/lib_var/chest0.so > $OUT/ab.txt 2>&1
echo rc=0
