#!/bin/bash
# Where the MAP kernel's time goes (run under gpurun from the repo root): the turbo-only bench with the kernel's
# diagnostic builds (MI355_TDEC_DIAG: 0 full, 1 backward pass only, 2 forward pass only, 3 backward without
# checkpoint stores, 4 backward loads only) -> "diag avg_MAP_launch_ms"
for d in 0 1 2 3 4; do
  MI355_TDEC_DIAG=$d timeout -k 10 300 python bench.py --workload tdec --steps 3 --warmup 1 --no-cpu "$@" \
    > gpurun_out/diag_$d.json 2>gpurun_out/diag_$d.err || exit 1
  python -c "import json,sys; r=json.load(open(sys.argv[1])); print('diag', sys.argv[2], r['roofline']['avg_launch_ms'])" \
    gpurun_out/diag_$d.json $d
done
