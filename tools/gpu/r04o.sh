#!/bin/bash
# r04o: latency kernel phase cycles with diagnostic variants (no state stores / no input reads / no normalisation)
set -e
OUT=gpurun_out/r04o
mkdir -p $OUT
export TMPDIR=/tmp LAT_PROBE_QUICK=1
for v in base latd1 latd2 latd4 latd7; do
  lib=srsran_amd/lib/libsrsran_amd.so; [ $v = base ] || lib=srsran_amd/lib_var/$v.so
  MI355_LIB=$lib timeout -k 10 120 python3 -u tools/lat_probe.py > $OUT/$v.jsonl 2> $OUT/$v.err
done
echo rc=0
