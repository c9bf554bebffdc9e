#!/bin/bash
# round 6: the driver's literal bench command at the final sources (PMC summaries keyed to them), then the same command
# under rocprofv3 --kernel-trace --stats (its kernel statistics for profiles/)
set -o pipefail
OUT=$PWD/gpurun_out/r06_drv
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], d['crc_ok_tbs'], r['frac'], r.get('traffic_frac'), r.get('avg_launch_ms'), d['dropin_tti_latency']['p50_ms'])"
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o drv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 \
  > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -30 $OUT/bench_prof.err; exit 1; }
echo rc=0
