#!/bin/bash
# r04x: configs[2] SISO QPSK with 2 / 3 / 4 find_and_decode chunks (host replay + PDSCH planning of chunk 0 left the
# GPU idle ~280 us per 8,192-subframe step with 2), twice each; kernel trace with the best
set -e
OUT=gpurun_out/r04x
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for c in 2 3 4; do
    MI355_UEDL_CHUNKS=$c timeout -k 10 300 python3 -u bench.py --workload siso_qpsk --steps 5 --warmup 2 --no-cpu --no-roofline > $OUT/siso_c$c.$rep.json 2> $OUT/siso_c$c.$rep.err
    python3 -c "import json,sys; r=json.load(open(sys.argv[1])); print(sys.argv[2], r['ms_per_step'], r['crc_ok_tbs'])" $OUT/siso_c$c.$rep.json c$c
  done
done
echo rc=0
