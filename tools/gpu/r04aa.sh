#!/bin/bash
# r04aa: latency kernel with single-DPP exchanges (group-lane relabelling) and the normalisation beside the step
set -e
OUT=gpurun_out/r04aa
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dlsch_gpu.py tests/test_dropin_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/dlsch.log 2>&1 || { rc=$?; echo dlsch rc=$rc; tail -30 $OUT/dlsch.log; exit $rc; }
timeout -k 10 300 python3 -u tools/lat_probe.py > $OUT/lat_probe.jsonl 2> $OUT/lat_probe.err
MI355_DLSCH_LAT_CBS=512 timeout -k 10 300 python3 -u tools/dropin_lat.py 500 > $OUT/dropin_lat_on.json 2> $OUT/dropin_lat_on.err
timeout -k 10 300 python3 -u tools/dropin_lat.py 500 > $OUT/dropin_lat_off.json 2> $OUT/dropin_lat_off.err
echo rc=0
