#!/bin/bash
# find_and_decode with 1 vs 2 control chunks (run under gpurun)
for c in 2 3 4 6 2 3 4 6; do
  MI355_UEDL_CHUNKS=$c timeout -k 10 300 python bench.py --workload ue_dl --no-cpu --no-waterfall --no-roofline > gpurun_out/uc.json 2>/dev/null || exit 1
  python -c "import json,sys; r=json.load(open('gpurun_out/uc.json')); print('chunks', sys.argv[1], r['ms_per_step'], r['crc_ok_tbs'])" $c
done
