#!/bin/bash
# r03z: CPU baseline with the reference-stage front end (default bench and siso_qpsk), drop-in latency included
set -e
OUT=gpurun_out/r03z
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 python -u bench.py --workload siso_qpsk > $OUT/siso.json 2> $OUT/siso.err
echo rc=0
