#!/bin/bash
# Step time of the bench workloads over PHY worker counts and find_and_decode chunks (run under gpurun):
#     tools/gpu/workers_ab.sh <tag> [reps=2]
# CFGS (env): "workload:workers:chunks ..." (chunks "-" = bench default); BENCH_STAGGER_MS passes through.
set -e
OUT=gpurun_out/$1; REPS=${2:-2}
mkdir -p $OUT
CFGS=${CFGS:-"pdsch:1:- pdsch:3:- ue_dl:3:1 ue_dl:3:2 siso_qpsk:3:1 siso_qpsk:2:1"}
for rep in $(seq 1 $REPS); do
  for cfg in $CFGS; do
    IFS=: read wl w c <<< "$cfg"
    ca=""; [ "$c" != "-" ] && ca="--chunks $c"
    f=$OUT/${wl}_w${w}_c${c}_$rep
    timeout -k 10 300 python3 bench.py --workload $wl --workers $w $ca --steps 20 --warmup 5 --no-cpu --no-waterfall \
      --no-roofline > $f.json 2> $f.err || { rc=$?; echo "$cfg rc=$rc"; tail -20 $f.err; exit $rc; }
    python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], r['ms_per_step'], r['value'], r['crc_ok_tbs'], r.get('payload_checked_tbs'), r.get('worker_calls'))" $f.json $cfg
  done
done
echo rc=0
