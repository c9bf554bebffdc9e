#!/bin/bash
# round 6 o4: what bounds the latency kernel's second parts with output waves: phase cycles with the output math off
# (LAT_DIAG 1) and with the output passes off (LAT_DIAG 2) -- timing only, wrong results
set -o pipefail
OUT=$PWD/gpurun_out/r06o4
mkdir -p $OUT
export TMPDIR=/tmp
for v in cur d1 d2; do
for ow in 1 0; do
  MI355_LAT_OWAVES=$ow MI355_LIB=srsran_amd/lib_var/$v.so LAT_PROBE_QUICK=1 timeout -k 10 300 python3 tools/lat_probe.py > $OUT/p_$v.json 2> $OUT/p_$v.err \
    || { tail -20 $OUT/p_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['us_per_call'], d['per_cb_half_it_kcycles'], d['load_kcycles_per_cb'])" $OUT/p_$v.json "$v owaves=$ow"
done
done
echo rc=0
