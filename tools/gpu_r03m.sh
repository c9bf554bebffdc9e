#!/bin/bash
# r03m: compact control read-back (hit records) + OFDM/estimation launched per find_and_decode chunk: control,
# ue_dl, chunk, drop-in, recorded-signal and matrix tests; ue_dl / pdsch bench; ue_dl timeline
set -e
OUT=gpurun_out/r03m
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_pdcch_gpu.py tests/test_ue_dl_gpu.py tests/test_uedl_chunks_gpu.py tests/test_dropin_gpu.py tests/test_real_signal.py tests/test_real_signal_10m.py tests/test_phy_dl_matrix_gpu.py tests/test_chest_state_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
timeout -k 10 300 python -u bench.py --workload ue_dl --no-cpu --no-waterfall --no-roofline > $OUT/ue_dl.json 2> $OUT/ue_dl.err
timeout -k 10 300 python -u bench.py --no-cpu --no-waterfall --no-roofline > $OUT/pdsch.json 2> $OUT/pdsch.err
timeout -k 10 300 python -u bench.py --workload ue_dl --no-cpu --no-waterfall --no-roofline > $OUT/ue_dl2.json 2> $OUT/ue_dl2.err
bash tools/trace_uedl.sh r03m
echo rc=0
