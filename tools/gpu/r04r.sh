#!/bin/bash
# r04r: latency kernel with pipelined output passes: DL-SCH + drop-in tests, probe, path crossover sweep, drop-in latency
set -e
OUT=gpurun_out/r04r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dlsch_gpu.py tests/test_dropin_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/dlsch.log 2>&1 || { rc=$?; echo dlsch rc=$rc; tail -30 $OUT/dlsch.log; exit $rc; }
timeout -k 10 300 python3 -u tools/lat_probe.py > $OUT/lat_probe.jsonl 2> $OUT/lat_probe.err
LAT_PROBE_SWEEP=1 timeout -k 10 300 python3 -u tools/lat_probe.py > $OUT/sweep.jsonl 2> $OUT/sweep.err
MI355_DLSCH_LAT_CBS=512 timeout -k 10 300 python3 -u tools/dropin_lat.py 500 > $OUT/dropin_lat_on.json 2> $OUT/dropin_lat_on.err
echo rc=0
