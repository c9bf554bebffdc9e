#!/bin/bash
# MAP kernel time against waves per CU (MI355_TDEC_LDS caps the resident workgroups of 4 waves):
# 0 -> register-limited (3 waves/SIMD), 60000 -> 2 workgroups/CU (2 waves/SIMD), 100000 -> 1 (1 wave/SIMD)
for lds in 0 60000 100000; do
  for d in 0 4; do
    MI355_TDEC_LDS=$lds MI355_TDEC_DIAG=$d timeout -k 10 300 python bench.py --workload tdec --steps 3 --warmup 1 --no-cpu "$@" \
      > gpurun_out/occ.json 2>gpurun_out/occ.err || exit 1
    python -c "import json,sys; r=json.load(open(sys.argv[1])); print('lds', sys.argv[2], 'diag', sys.argv[3], r['roofline']['avg_launch_ms'])" \
      gpurun_out/occ.json $lds $d
  done
done
