#!/bin/bash
# r03k: drop-in TTI latency with power scaling, ue_dl timeline with host phase timing
set -e
OUT=gpurun_out/r03k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_dropin_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu --no-waterfall > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 python -u bench.py --workload ue_dl --no-cpu --no-waterfall --no-roofline > $OUT/ue_dl.json 2> $OUT/ue_dl.err
bash tools/trace_uedl.sh r03k
echo rc=0
