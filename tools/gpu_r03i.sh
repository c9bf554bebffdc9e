#!/bin/bash
# r03i: control read-backs on a copy stream: control tests, ue_dl bench (2 and 3 chunks) + trace
set -e
OUT=gpurun_out/r03i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_pdcch_gpu.py tests/test_real_signal.py tests/test_real_signal_10m.py tests/test_dropin_gpu.py tests/test_uedl_chunks_gpu.py tests/test_phy_dl_matrix_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
timeout -k 10 300 python -u bench.py --workload ue_dl --no-cpu --no-waterfall --no-roofline > $OUT/ue_dl.json 2> $OUT/ue_dl.err
MI355_UEDL_CHUNKS=3 timeout -k 10 300 python -u bench.py --workload ue_dl --no-cpu --no-waterfall --no-roofline > $OUT/ue_dl3.json 2> $OUT/ue_dl3.err
timeout -k 10 300 python -u bench.py --no-cpu --no-waterfall --no-roofline > $OUT/pdsch.json 2> $OUT/pdsch.err
bash tools/trace_uedl.sh r03i
echo rc=0
