#!/bin/bash
# r03op: OFDM demodulator LDS padding after the first radix-8 stage -- OFDM / ue_dl / real-signal parity, A/B against
# the unpadded layout (srsran_amd/lib_var/ofdmpad0.so, -DOFDM_PAD=0)
set -e
OUT=gpurun_out/r03op
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_real_signal.py tests/test_real_signal_10m.py tests/test_ue_dl_gpu.py tests/test_enb_dl_gpu.py tests/test_dropin_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
KF=ofdm_rx,chest_estimate bash tools/gpu_eqk.sh srsran_amd/lib/libsrsran_amd.so srsran_amd/lib_var/ofdmpad0.so srsran_amd/lib/libsrsran_amd.so srsran_amd/lib_var/ofdmpad0.so > $OUT/ab.txt 2>&1
echo rc=0
