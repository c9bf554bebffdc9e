#!/bin/bash
# round 6, final sources: the closing phases (GPU suite, smoke, the driver's bench command, secondary workloads, e2e
# kernel statistics), then the latency kernel's phase cycles and the drop-in per-TTI latency with and without the
# output waves
set -o pipefail
TAG=${1:-r06_final}
bash tools/gpu/closing.sh $TAG suite smoke driver workloads e2estats || exit 1
OUT=$PWD/gpurun_out/$TAG
for ow in 0 1; do
  MI355_LAT_OWAVES=$ow LAT_PROBE_QUICK=1 timeout -k 10 300 python3 tools/lat_probe.py > $OUT/probe_$ow.json 2> $OUT/probe_$ow.err \
    || { tail -20 $OUT/probe_$ow.err; exit 1; }
  echo "probe owaves=$ow $(tail -c 500 $OUT/probe_$ow.json)"
done
for ow in 0 1 0 1; do
  MI355_LAT_OWAVES=$ow timeout -k 10 300 python3 tools/dropin_lat.py 1000 > $OUT/d_$ow.json 2> $OUT/d_$ow.err || { tail -20 $OUT/d_$ow.err; exit 1; }
  python3 -c "import json,sys; e=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('owaves', sys.argv[2], 'p50', e['p50_ms'], 'p99', e['p99_ms'], 'max', e['max_ms'], e['stage_p50_ms'], e['tbs_ok'])" $OUT/d_$ow.json $ow
done
echo rc=0
