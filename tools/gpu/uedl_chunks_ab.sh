#!/bin/bash
# find_and_decode chunks (MI355_UEDL_CHUNKS) x PHY workers on the ue_dl workload (run under gpurun)
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
for rep in 1 2; do
  for cw in "2 2" "1 2" "1 3" "2 3"; do
    set -- $cw
    MI355_UEDL_CHUNKS=$1 timeout -k 10 300 python3 bench.py --workload ue_dl --workers $2 --steps 20 --warmup 3 --no-cpu --no-waterfall --no-roofline > $OUT/c$1_w$2_$rep.json 2> $OUT/c$1_w$2_$rep.err
    python3 -c "import json,sys; r=json.load(open(sys.argv[1])); print('chunks', sys.argv[2], 'workers', sys.argv[3], r['ms_per_step'], r['value'], r['crc_ok_tbs'], r['payload_checked_tbs'])" $OUT/c$1_w$2_$rep.json $1 $2
  done
done
echo rc=0
