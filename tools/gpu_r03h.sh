#!/bin/bash
# r03h: blind decoder with one wave per workgroup: control tests, ue_dl bench + trace
set -e
OUT=gpurun_out/r03h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_pdcch_gpu.py tests/test_real_signal.py tests/test_real_signal_10m.py tests/test_dropin_gpu.py tests/test_uedl_chunks_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
timeout -k 10 300 python -u bench.py --workload ue_dl --no-cpu --no-waterfall > $OUT/ue_dl.json 2> $OUT/ue_dl.err
bash tools/trace_uedl.sh r03h
echo rc=0
