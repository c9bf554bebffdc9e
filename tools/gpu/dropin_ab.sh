#!/bin/bash
# Drop-in per-TTI latency A/B of an environment setting on one box:  tools/gpu/dropin_ab.sh <tag> "<ENV=a>" "<ENV=b>" [reps=3]
set -e
OUT=gpurun_out/$1; A=$2; B=$3; REPS=${4:-3}; mkdir -p $OUT
for rep in $(seq 1 $REPS); do
  for v in "$A" "$B"; do
    f=$OUT/$(echo "$v" | tr -c 'A-Za-z0-9_' '_')_$rep.json
    env $v timeout -k 10 300 python3 -u tools/dropin_lat.py 1000 > $f 2> $f.err || { rc=$?; tail -20 $f.err; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['p50_ms'], d['p99_ms'], d['stage_p50_ms'], d['tbs_ok'])" $f "$v"
  done
done
