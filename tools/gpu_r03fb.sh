#!/bin/bash
# r03f (part B): benches (default with CPU baseline and MAP traffic, ue_dl, tdec, siso_qpsk) and kernel statistics
set -e
OUT=gpurun_out/r03f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --workload ue_dl --no-cpu --no-waterfall > $OUT/ue_dl.json 2> $OUT/ue_dl.err
timeout -k 10 300 python -u bench.py --workload tdec > $OUT/tdec.json 2> $OUT/tdec.err
timeout -k 10 300 python -u bench.py --workload siso_qpsk > $OUT/siso.json 2> $OUT/siso.err
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
bash tools/gpu_stats.sh r03f > /dev/null
echo rc=0
