#!/bin/bash
# r04h: configs[2] SISO QPSK batch size (per-subframe time at 2,048 / 4,096 / 8,192 subframes per step: the MAP
# launch of a 2,048-subframe chunk has only 384 waves); find_and_decode vs pdsch on one box (item 5), twice each
set -e
OUT=gpurun_out/r04h
mkdir -p $OUT
export TMPDIR=/tmp
for n in 2048 4096 8192; do
  timeout -k 10 300 python3 -u bench.py --workload siso_qpsk --subframes $n --steps 5 --warmup 2 --no-cpu --no-roofline > $OUT/siso_$n.json 2> $OUT/siso_$n.err
done
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --workload pdsch --steps 10 --warmup 3 --no-cpu --no-waterfall --no-roofline > $OUT/pdsch_$i.json 2> $OUT/pdsch_$i.err
  timeout -k 10 300 python3 -u bench.py --workload ue_dl --steps 10 --warmup 3 --no-cpu --no-waterfall --no-roofline > $OUT/ue_dl_$i.json 2> $OUT/ue_dl_$i.err
done
echo rc=0
