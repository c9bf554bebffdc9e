#!/bin/bash
# A/B/C timing of MAP-kernel builds: tools/ab3.sh <lib>... -- prints "<lib> tdec:<avg MAP ms> e2e:<ms/step> <MAP ms>"
set -o pipefail
for rep in 1 2; do
for lib in "$@"; do
  MI355_LIB=$lib timeout -k 10 200 python bench.py --workload tdec --steps 3 --warmup 1 --no-cpu > gpurun_out/ab_t.json 2>/dev/null || exit 1
  MI355_LIB=$lib timeout -k 10 200 python bench.py --no-cpu --no-waterfall --steps 5 > gpurun_out/ab_e.json 2>/dev/null || exit 1
  python -c "
import json,sys
t=json.load(open('gpurun_out/ab_t.json')); e=json.load(open('gpurun_out/ab_e.json'))
print(sys.argv[1], 'tdec', t['roofline']['avg_launch_ms'], 'e2e', e['ms_per_step'], e['roofline']['avg_launch_ms'], e['crc_ok_tbs'])" $lib
done
done
