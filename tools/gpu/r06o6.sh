#!/bin/bash
# round 6 o6: the latency kernel's second parts with output waves but no handoff at all (LAT_DIAG 6: no passes, no
# waits or posts; timing only) against no passes with the handoff (LAT_DIAG 2) and the real kernel
set -o pipefail
OUT=$PWD/gpurun_out/r06o6
mkdir -p $OUT
export TMPDIR=/tmp
for v in cur d2 d6; do
for ow in 1 0; do
  MI355_LAT_OWAVES=$ow MI355_LIB=srsran_amd/lib_var/$v.so LAT_PROBE_QUICK=1 timeout -k 10 300 python3 tools/lat_probe.py > $OUT/p_$v.json 2> $OUT/p_$v.err \
    || { tail -20 $OUT/p_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['us_per_call'], d['per_cb_half_it_kcycles'])" $OUT/p_$v.json "$v owaves=$ow"
done
done
echo rc=0
