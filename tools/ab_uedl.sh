#!/bin/bash
# A/B of two in-tree library builds on one box (run under gpurun), e2e and find_and_decode:
#   tools/ab_uedl.sh <A.so> <B.so>  ->  "<lib> pdsch_ms ue_dl_ms" for A, B, A, B
A=$1; B=$2
mkdir -p gpurun_out/ab
for lib in $A $B $A $B; do
  MI355_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --no-waterfall --no-roofline > gpurun_out/ab/p.json 2>gpurun_out/ab/p.err || exit 1
  MI355_LIB=$lib timeout -k 10 300 python bench.py --workload ue_dl --no-cpu --no-waterfall --no-roofline > gpurun_out/ab/u.json 2>gpurun_out/ab/u.err || exit 1
  python -c "import json,sys; p=json.load(open('gpurun_out/ab/p.json')); u=json.load(open('gpurun_out/ab/u.json')); print(sys.argv[1], p['ms_per_step'], u['ms_per_step'], p['crc_ok_tbs'], u['crc_ok_tbs'])" $lib
done
