#!/bin/bash
# r04n: latency kernel SIMD placement: probe with two-wave and four-wave workgroups, drop-in latency with each
set -e
OUT=gpurun_out/r04n
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dlsch_gpu.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/dlsch.log 2>&1 || { rc=$?; echo dlsch rc=$rc; [ $rc -eq 1 ] || exit $rc; }
MI355_LAT_WAVES=4 timeout -k 10 300 python -u -m pytest tests/test_dlsch_gpu.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/dlsch4.log 2>&1 || { rc=$?; echo dlsch4 rc=$rc; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 300 python3 -u tools/lat_probe.py > $OUT/lat_probe2.jsonl 2> $OUT/lat_probe2.err
MI355_LAT_WAVES=4 timeout -k 10 300 python3 -u tools/lat_probe.py > $OUT/lat_probe4.jsonl 2> $OUT/lat_probe4.err
MI355_DLSCH_LAT_CBS=512 timeout -k 10 300 python3 -u tools/dropin_lat.py 500 > $OUT/dropin_lat_on2.json 2> $OUT/dropin_lat_on2.err
MI355_LAT_WAVES=4 MI355_DLSCH_LAT_CBS=512 timeout -k 10 300 python3 -u tools/dropin_lat.py 500 > $OUT/dropin_lat_on4.json 2> $OUT/dropin_lat_on4.err
echo rc=0
