#!/bin/bash
# r04s: latency kernel second-part split (no output computation / no passes), path crossover sweep, drop-in latency
set -e
OUT=gpurun_out/r04s
mkdir -p $OUT
export TMPDIR=/tmp
for v in latd1 latd2; do
  LAT_PROBE_QUICK=1 MI355_LIB=srsran_amd/lib_var/$v.so timeout -k 10 120 python3 -u tools/lat_probe.py > $OUT/$v.jsonl 2> $OUT/$v.err
done
LAT_PROBE_SWEEP=1 timeout -k 10 300 python3 -u tools/lat_probe.py > $OUT/sweep.jsonl 2> $OUT/sweep.err
MI355_DLSCH_LAT_CBS=512 timeout -k 10 300 python3 -u tools/dropin_lat.py 500 > $OUT/dropin_lat_on.json 2> $OUT/dropin_lat_on.err
echo rc=0
