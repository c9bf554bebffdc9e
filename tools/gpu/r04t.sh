#!/bin/bash
# r04t: DL-SCH path crossover sweep (latency vs throughput path by transport blocks per call)
set -e
OUT=gpurun_out/r04t
mkdir -p $OUT
export TMPDIR=/tmp
LAT_PROBE_SWEEP=1 timeout -k 10 300 python3 -u tools/lat_probe.py > $OUT/sweep.jsonl 2> $OUT/sweep.err
echo rc=0
