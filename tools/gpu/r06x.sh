#!/bin/bash
# round 6 x: the default step (configs[3], 3 PHY workers) of the round-5 tree (ab_r05/, cd7eba4 with its own library,
# not committed) vs HEAD on one box, alternating; then the one-worker step and kernel statistics of each
set -o pipefail
OUT=$PWD/gpurun_out/r06x
mkdir -p $OUT
export TMPDIR=/tmp
for t in r05 head r05 head; do
  d=.; [ $t = r05 ] && d=ab_r05
  (cd $d && timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-waterfall --no-roofline \
    > $OUT/p_$t.json 2> $OUT/p_$t.err) || { tail -20 $OUT/p_$t.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['worker_calls'], d.get('stage_ms'), d['crc_ok_tbs'])" $OUT/p_$t.json $t
done
for t in r05 head; do
  d=.; [ $t = r05 ] && d=ab_r05
  (cd $d && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/k_$t -o k -- python3 bench.py \
    --workers 1 --steps 5 --warmup 2 --no-cpu --no-waterfall --no-roofline > $OUT/k_$t.json 2> $OUT/k_$t.err) \
    || { tail -20 $OUT/k_$t.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '1 worker (profiled)', d['ms_per_step'])" $OUT/k_$t.json $t
done
echo rc=0
