#!/bin/bash
# find_and_decode with the first of two chunks at different shares (MI355_UEDL_SPLIT0, percent): "<pct> ue_dl_ms"
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for pct in 50 42 35 28; do
    MI355_UEDL_SPLIT0=$pct timeout -k 10 300 python bench.py --workload ue_dl --no-cpu --no-waterfall --no-roofline > gpurun_out/ab/s.json 2>gpurun_out/ab/s.err || exit 1
    python -c "import json,sys; u=json.load(open('gpurun_out/ab/s.json')); print(sys.argv[1], u['ms_per_step'], u['crc_ok_tbs'])" $pct
  done
done
timeout -k 10 300 python bench.py --no-cpu --no-waterfall --no-roofline > gpurun_out/ab/p.json 2>gpurun_out/ab/p.err || exit 1
python -c "import json; p=json.load(open('gpurun_out/ab/p.json')); print('pdsch', p['ms_per_step'])"
