#!/bin/bash
# The driver's literal bench command N times back to back on one box (run-to-run spread of the headline):
#     tools/gpu/driver_rep.sh <tag> [N=3] [extra bench args, e.g. --workers 1]
# gpurun_out/<tag>/driver_<i>.json; prints ms_per_step, value and the timed calls' p50 / max per run.
set -e
TAG=${1:?tag}; N=${2:-3}; shift; shift || true; EXTRA="$*"
OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in $(seq 1 $N); do
  timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 $EXTRA > $OUT/driver_$i.json 2> $OUT/driver_$i.err \
    || { rc=$?; echo "run $i rc=$rc"; tail -30 $OUT/driver_$i.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$OUT/driver_$i.json').read().strip().splitlines()[-1]); \
print('run $i $EXTRA', d['ms_per_step'], d['value'], d['crc_ok_tbs'], d.get('worker_calls'), d['roofline']['avg_launch_ms'])"
done
