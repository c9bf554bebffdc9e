#!/bin/bash
# round 6 u: SISO QPSK (configs[2]) at HEAD vs the round-5 tree (ab_r05/: cd7eba4 with its own library, not
# committed), same box, alternating: bench steps, then one-worker kernel statistics of each
set -o pipefail
OUT=$PWD/gpurun_out/r06u
mkdir -p $OUT
export TMPDIR=/tmp
for t in r05 head r05 head; do
  d=.; [ $t = r05 ] && d=ab_r05
  (cd $d && timeout -k 10 300 python3 bench.py --workload siso_qpsk --steps 10 --warmup 3 --no-cpu --no-waterfall \
    --no-roofline > $OUT/siso_$t.json 2> $OUT/siso_$t.err) || { tail -20 $OUT/siso_$t.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['worker_calls'], d['crc_ok_tbs'])" $OUT/siso_$t.json $t
done
for t in r05 head; do
  d=.; [ $t = r05 ] && d=ab_r05
  (cd $d && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/k_$t -o k -- python3 bench.py \
    --workload siso_qpsk --workers 1 --steps 3 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/k_$t.json 2> $OUT/k_$t.err) \
    || { tail -20 $OUT/k_$t.err; exit 1; }
done
echo rc=0
