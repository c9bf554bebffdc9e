#!/bin/bash
# A/B of the e2e waterfall field (EPA 28 dB: real work in the later half-iterations):  tools/ab_wf.sh <A.so> <B.so>
A=$1; B=$2
mkdir -p gpurun_out/ab
for lib in $A $B $A $B; do
  MI355_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --no-roofline --steps 2 --warmup 1 > gpurun_out/ab/w.json 2>gpurun_out/ab/w.err || exit 1
  python -c "import json,sys; r=json.load(open('gpurun_out/ab/w.json')); w=r['e2e_waterfall']; print(sys.argv[1], r['ms_per_step'], w['ms_per_step'], w['crc_ok_tbs'])" $lib
done
