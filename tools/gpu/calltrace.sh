#!/bin/bash
# PHY-worker call timelines of the default workload (BENCH_CALL_TRACE), to find host-side stalls in the timed region:
#     tools/gpu/calltrace.sh <tag> "<workers list>" [extra bench args]
set -e
TAG=${1:?tag}; WL=${2:-"3 3 2 1"}; shift; shift || true; EXTRA="$*"
OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
cgs() { cat /sys/fs/cgroup/cpu.stat 2>/dev/null | tr '\n' ' '; }
echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null) nproc $(nproc)"
for w in $WL; do
  echo "before: $(cgs)"
  i=$((i+1))
  BENCH_CALL_TRACE=$OUT/trace_${i}_w$w.json timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 \
    --workers $w --no-cpu --no-roofline --no-waterfall $EXTRA > $OUT/b_${i}_w$w.json 2> $OUT/b_${i}_w$w.err \
    || { rc=$?; echo "run $i rc=$rc"; tail -30 $OUT/b_${i}_w$w.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$OUT/b_${i}_w$w.json').read().strip().splitlines()[-1]); \
print('run $i workers $w', d['ms_per_step'], d['value'], d['crc_ok_tbs'], d.get('worker_calls'))"
  echo "after:  $(cgs)"
done
