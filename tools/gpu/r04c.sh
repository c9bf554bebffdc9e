#!/bin/bash
# r04c: after the row-mask LDS fix (words of missing / finished code blocks were read uninitialised) and with the
# DL-SCH latency path (tdec_win_lat): DL-SCH / turbo tests first, then the GPU suite, bench, drop-in latency trace
set -e
OUT=gpurun_out/r04c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dlsch_gpu.py tests/test_tdec_gpu.py tests/test_srslte_tdec_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/first.log 2>&1 || { rc=$?; echo first rc=$rc; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_suite.log 2>&1 || { rc=$?; echo suite rc=$rc; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 400 python3 -u bench.py --no-waterfall > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/lat -o lat -- python3 tools/dropin_lat.py 200 > $OUT/lat.log 2>&1
echo rc=0
