#!/bin/bash
# round 6: the driver's weak-scaling command at N = 8, rehearsed with the 8 ranks sharing the one GPU of a test box
# (gloo collectives; RCCL refuses two ranks on one device): launcher, barriers, max-over-ranks time, CRC-bitmap gather
set -o pipefail
OUT=$PWD/gpurun_out/r06n8
mkdir -p $OUT
export TMPDIR=/tmp
(for i in $(seq 1 40); do date +%T >> $OUT/tick; sleep 20; done) &
TK=$!
BENCH_DIST_BACKEND=gloo BENCH_SHARE_GPU=1 timeout -k 10 700 python3 -u bench.py --gpus 8 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?
kill $TK
echo rc=$rc
tail -c 1500 $OUT/bench.json
exit $rc
