#!/bin/bash
# A/B of two in-tree library builds on one box (run under gpurun): tools/ab_lib.sh <A.so> <B.so> [bench args...]
# prints "<lib> e2e_ms MAP_avg_ms fixed8_ms" for A, B, A, B
A=$1; B=$2; shift 2
mkdir -p gpurun_out/ab
for lib in $A $B $A $B; do
  MI355_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --no-waterfall "$@" > gpurun_out/ab/ab.json 2>gpurun_out/ab/ab.err || exit 1
  python -c "import json,sys; r=json.load(open('gpurun_out/ab/ab.json')); print(sys.argv[1], r['ms_per_step'], r['roofline']['avg_launch_ms'], r.get('decoder_bound_fixed8', {}).get('ms'))" $lib
done
