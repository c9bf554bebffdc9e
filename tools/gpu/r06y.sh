#!/bin/bash
# round 6 y: --workload ue_dl and the drop-in per-TTI latency loop of the round-5 tree (ab_r05/, not committed) vs
# HEAD on one box, alternating
set -o pipefail
OUT=$PWD/gpurun_out/r06y
mkdir -p $OUT
export TMPDIR=/tmp
for t in r05 head r05 head; do
  d=.; [ $t = r05 ] && d=ab_r05
  (cd $d && timeout -k 10 300 python3 bench.py --workload ue_dl --steps 10 --warmup 3 --no-cpu --no-waterfall --no-roofline \
    > $OUT/u_$t.json 2> $OUT/u_$t.err) || { tail -20 $OUT/u_$t.err; exit 1; }
  (cd $d && timeout -k 10 300 python3 tools/dropin_lat.py 1000 > $OUT/d_$t.json 2> $OUT/d_$t.err) || { tail -20 $OUT/d_$t.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); print(sys.argv[3], 'ue_dl', d['ms_per_step'], d['crc_ok_tbs'], '| dropin p50', e['p50_ms'], 'p99', e['p99_ms'], 'max', e['max_ms'], e['stage_p50_ms'], e['tbs_ok'])" $OUT/u_$t.json $OUT/d_$t.json $t
done
echo rc=0
