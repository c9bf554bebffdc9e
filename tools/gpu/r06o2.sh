#!/bin/bash
# round 6 o2: the latency turbo kernel's output passes on two more waves (A.owaves, MI355_LAT_OWAVES) -- DL-SCH (both
# turbo paths) / drop-in / tdec API GPU parity, the kernel's phase cycles (tools/lat_probe.py, quick case) and the
# drop-in per-TTI latency, owaves 0 vs 1 alternating
set -o pipefail
OUT=$PWD/gpurun_out/r06o2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_dlsch_gpu.py tests/test_dropin_gpu.py tests/test_srslte_tdec_gpu.py \
  tests/test_dlsch8_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 \
  || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for ow in 0 1; do
  MI355_LAT_OWAVES=$ow LAT_PROBE_QUICK=1 timeout -k 10 300 python3 tools/lat_probe.py > $OUT/probe_$ow.json 2> $OUT/probe_$ow.err \
    || { tail -20 $OUT/probe_$ow.err; exit 1; }
  echo "probe owaves=$ow $(tail -c 700 $OUT/probe_$ow.json)"
done
for ow in 0 1 0 1; do
  MI355_LAT_OWAVES=$ow timeout -k 10 300 python3 tools/dropin_lat.py 1000 > $OUT/d_$ow.json 2> $OUT/d_$ow.err || { tail -20 $OUT/d_$ow.err; exit 1; }
  python3 -c "import json,sys; e=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('owaves', sys.argv[2], 'p50', e['p50_ms'], 'p99', e['p99_ms'], 'max', e['max_ms'], e['stage_p50_ms'], e['tbs_ok'])" $OUT/d_$ow.json $ow
done
echo rc=0
