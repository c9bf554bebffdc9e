#!/bin/bash
# Step time of the pdsch / ue_dl workloads with 1, 2, 3 PHY worker threads (run under gpurun): tools/gpu/workers_ab.sh <tag>
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
for rep in 1 2; do
  for wl in ${WLS:-pdsch ue_dl}; do
    for w in 1 2 3; do
      timeout -k 10 300 python3 bench.py --workload $wl --workers $w --steps 20 --warmup 3 --no-cpu --no-waterfall --no-roofline > $OUT/${wl}_w${w}_$rep.json 2> $OUT/${wl}_w${w}_$rep.err
      python3 -c "import json,sys; r=json.load(open(sys.argv[1])); print(sys.argv[2], 'workers', sys.argv[3], r['ms_per_step'], r['value'], r['crc_ok_tbs'], r['payload_checked_tbs'])" $OUT/${wl}_w${w}_$rep.json $wl $w
    done
  done
done
echo rc=0
