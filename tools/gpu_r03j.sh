#!/bin/bash
# r03j: drop-in per-TTI latency (caller_tti_latency) test + full default bench (dropin_tti_latency field)
set -e
OUT=gpurun_out/r03j
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_dropin_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
echo rc=0
