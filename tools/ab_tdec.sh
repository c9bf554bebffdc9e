#!/bin/bash
# A/B timing of two in-tree library builds on one box: tools/ab_tdec.sh <A.so> <B.so> [bench args...]
# prints "<lib> ms_per_step avg_MAP_launch_ms" for A, B, A, B (interleaved against drift)
A=$1; B=$2; shift 2
for lib in $A $B $A $B; do
  MI355_LIB=$lib timeout -k 10 300 python bench.py --no-cpu "$@" > gpurun_out/ab.json 2>/dev/null || exit 1
  python -c "import json,sys; r=json.load(open('gpurun_out/ab.json')); print(sys.argv[1], r['ms_per_step'], r['roofline']['avg_launch_ms'])" $lib
done
