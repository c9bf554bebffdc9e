#!/bin/bash
# round 6 o5: latency kernel with output waves -- which SIMDs they share, and the recursion waves at a higher issue
# priority (LAT_PRIO), with and without sleeping polls: tools/lat_probe.py phase cycles, two rounds
set -o pipefail
OUT=$PWD/gpurun_out/r06o5
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
for v in cur prio prio_sleep; do
  MI355_LIB=srsran_amd/lib_var/$v.so LAT_PROBE_QUICK=1 timeout -k 10 300 python3 tools/lat_probe.py > $OUT/p_$v.json 2> $OUT/p_$v.err \
    || { tail -20 $OUT/p_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['us_per_call'], d['per_cb_half_it_kcycles'], d['simd'], d['rets'])" $OUT/p_$v.json $v
done
done
echo rc=0
