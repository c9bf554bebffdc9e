#!/bin/bash
# Where the MAP schedule's time goes: the bandwidth-only clone with parts of its traffic removed (variant builds,
# tools/build_variant.sh <name> -DTDEC_CLONE_NO_*=1), timed by the default bench's MAP probe (pool buffers with the
# parity-row bitmaps) and by the tdec workload (full parity):  tools/gpu/clone_ab.sh <tag> <lib.so> ...
# prints "<lib> e2e: real_ms clone_ms | tdec: real_ms clone_ms"
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for lib in "$@"; do
  n=$(basename $lib .so)
  MI355_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu --no-waterfall --steps 3 --warmup 1 > $OUT/e_$n.json 2> $OUT/e_$n.err
  MI355_LIB=$lib timeout -k 10 300 python3 bench.py --workload tdec --no-cpu --steps 3 --warmup 1 > $OUT/t_$n.json 2> $OUT/t_$n.err
  python3 -c "import json,sys; e=json.load(open(sys.argv[1]))['roofline']; t=json.load(open(sys.argv[2]))['roofline']; print(sys.argv[3], 'e2e:', e['avg_launch_ms'], e.get('schedule_clone_ms'), '| tdec:', t['avg_launch_ms'], t.get('schedule_clone_ms'))" $OUT/e_$n.json $OUT/t_$n.json $n
done
echo rc=0
