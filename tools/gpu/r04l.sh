#!/bin/bash
# r04l: latency kernel with batched output passes (64 lanes per pass): DL-SCH + drop-in tests, probe, drop-in latency
set -e
OUT=gpurun_out/r04l
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dlsch_gpu.py tests/test_dropin_gpu.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/dlsch.log 2>&1 || { rc=$?; echo dlsch rc=$rc; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 300 python3 -u tools/lat_probe.py > $OUT/lat_probe.jsonl 2> $OUT/lat_probe.err || { rc=$?; echo probe rc=$rc; [ $rc -eq 1 ] || exit $rc; }
MI355_DLSCH_LAT_CBS=512 timeout -k 10 300 python3 -u tools/dropin_lat.py 500 > $OUT/dropin_lat_on.json 2> $OUT/dropin_lat_on.err
timeout -k 10 300 python3 -u tools/dropin_lat.py 500 > $OUT/dropin_lat_off.json 2> $OUT/dropin_lat_off.err
echo rc=0
